# GPU op + train tests, the bench line, and a kernel trace of 5 bench steps.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-q2}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' $O/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1
echo "prof rc $?"
