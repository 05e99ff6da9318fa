# parity tests (default mode) then A/B of halo pipeline modes on layers and on the step
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
for m in 0 2; do
  TPG_HALO_MODE=$m timeout -k 10 200 python -u tools/bench_layers.py --iters 10 --passes fwd,dgrad --only enhance_128,add_128,conv0_res,conv5_0,enhance_64,add_64,enhance_32,enhance_16,conv4_res,local_40 > $O/layers_m$m.log 2>&1
done
for m in 0 -1; do
  TPG_HALO_MODE=$m timeout -k 10 200 python -u bench.py --steps 15 --warmup 4 --no-cpu-baseline > $O/bench_m$m.log 2>&1
done
echo done
