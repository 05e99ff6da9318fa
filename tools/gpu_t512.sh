cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-t512}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -k "512 or conv_vs_oracle or fused_backward" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/bench_layers.py --only add_128,conv0_res,conv5_0,add_64,local_40 > $O/layers.log 2>&1 || exit 1
TPG_HALO_NO512=1 timeout -k 10 200 python3 -u tools/bench_layers.py --only add_128,conv0_res,conv5_0 --passes fwd,dgrad > $O/layers256.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
TPG_HALO_NO512=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench256.log 2>&1
echo "bench rc $?"; cat $O/layers.log $O/layers256.log | grep -v amdgpu; grep -ho '"ms_per_step": [0-9.]*' $O/bench.log $O/bench256.log
