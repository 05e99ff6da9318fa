cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pf}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
L=enhance_128,e128_nores,add_128,conv0_res,enhance_64,enhance_32
timeout -k 10 200 python3 -u tools/bench_layers.py --only $L --passes fwd > $O/la.log 2>&1 || exit 1
TPG_HALO_VAR=32 timeout -k 10 200 python3 -u tools/bench_layers.py --only $L --passes fwd > $O/lb.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/ba.log 2>&1 &&
TPG_HALO_VAR=32 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bb.log 2>&1
echo "bench rc $?"; cat $O/la.log $O/lb.log | grep -v amdgpu; grep -ho '"ms_per_step": [0-9.]*' $O/ba.log $O/bb.log
