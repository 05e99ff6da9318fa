# Parity suite, then per-layer + step A/B of an env switch set vs unset (2 interleaved rounds).
#   bash tools/gpu_ab_env.sh TAG VAR layer1,layer2,...
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; VAR=$2; L=$3
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_all.log 2>&1
for rep in 1 2; do
  for v in 0 1; do
    if [ $v = 1 ]; then export $VAR=1; else unset $VAR; fi
    timeout -k 10 200 python -u tools/bench_layers.py --iters 10 --passes fwd,dgrad --only $L > $O/layers_set$v.r$rep.log 2>&1
    timeout -k 10 200 python -u bench.py --steps 15 --warmup 4 --no-cpu-baseline > $O/bench_set$v.r$rep.log 2>&1
  done
done
echo done
