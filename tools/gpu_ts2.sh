cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ts2}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
L=${LAYERS:-conv1_s2,conv2_s2,conv3_s2,conv4_s2,d_conv1_s2,up_128}
timeout -k 10 200 python3 -u tools/bench_layers.py --only $L --passes fwd,dgrad > $O/layers.log 2>&1 || exit 1
env ${ENVB:-TPG_HALO_NO_S2=1} timeout -k 10 200 python3 -u tools/bench_layers.py --only $L --passes fwd,dgrad > $O/layers_igemm.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
env ${ENVB:-TPG_HALO_NO_S2=1} timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_igemm.log 2>&1
echo "bench rc $?"; cat $O/layers.log $O/layers_igemm.log | grep -v amdgpu; grep -ho '"ms_per_step": [0-9.]*' $O/bench.log $O/bench_igemm.log
