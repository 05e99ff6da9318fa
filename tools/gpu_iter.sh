# Kernel iteration call: conv parity tests, per-layer microbench, train-step bench.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-it}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -u tools/bench_layers.py --iters 10 --only ${2:-enhance_128,add_128,conv0_res,conv5_0,enhance_64,add_64,enhance_32,enhance_16,enh_8,conv4_res,local_40,local_20} > $O/layers.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1
echo done
