cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-dil}; mkdir -p $O
L=conv2_s2,d_conv1_s2,up_64,up_32,conv1_s2
timeout -k 10 200 python3 -u tools/bench_layers.py --only $L --passes fwd,dgrad > $O/l32.log 2>&1 || exit 1
TPG_DILATED_MAXPIX=4096 timeout -k 10 200 python3 -u tools/bench_layers.py --only $L --passes fwd,dgrad > $O/l64.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/b32.log 2>&1 &&
TPG_DILATED_MAXPIX=4096 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/b64.log 2>&1
echo "bench rc $?"; cat $O/l32.log $O/l64.log | grep -v amdgpu; grep -ho '"ms_per_step": [0-9.]*' $O/b32.log $O/b64.log
