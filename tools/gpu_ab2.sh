# Quick parity (ops + model) then per-layer A/B of halo pipeline variants (TPG_HALO_VAR).
#   bash tools/gpu_ab2.sh TAG "VAR_A VAR_B ..." [layers]
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
L=${3:-enhance_128,add_128,conv0_res,conv5_0,enhance_64,add_64,enhance_32,enhance_16,conv4_res,local_40}
for v in $2; do
  TPG_HALO_VAR=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_v$v.log 2>&1
done
for rep in 1 2; do
  for v in $2; do
    TPG_HALO_VAR=$v timeout -k 10 200 python -u tools/bench_layers.py --iters 10 --passes fwd,dgrad --only $L > $O/layers_v${v}_r$rep.log 2>&1
  done
done
echo done
