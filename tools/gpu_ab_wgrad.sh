# Weight-gradient layer timings and the train step with the row/image-halo default on (1) / off (0).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
L=${2:-conv4_res,enh_8,enhance_16,enhance_32,enhance_64,local_10,local_20}
for rep in 1 2; do
  for v in 1 0; do
    TPG_WGRAD_RH=$v timeout -k 10 200 python -u tools/bench_layers.py --iters 10 --passes wgrad --only $L > $O/layers_rh$v.r$rep.log 2>&1
  done
  timeout -k 10 200 python -u bench.py --steps 15 --warmup 4 --no-cpu-baseline > $O/bench.r$rep.log 2>&1
done
echo done
