# A/B of an env switch on the per-layer microbench (same box, back to back).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-ab}; VAR=$2; A=$3; B=$4; L=${5:-enhance_128,add_128,conv0_res,conv5_0,enhance_64,enhance_32,enhance_16}
O=gpurun_out/$T; mkdir -p $O
for rep in 1 2; do
  env $VAR=$A timeout -k 10 200 python -u tools/bench_layers.py --iters 10 --only $L > $O/A$rep.log 2>&1
  env $VAR=$B timeout -k 10 200 python -u tools/bench_layers.py --iters 10 --only $L > $O/B$rep.log 2>&1
done
echo done
