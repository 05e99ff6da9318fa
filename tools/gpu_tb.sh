# Full GPU suite, then two default bench lines (no CPU baseline) with the tuning dump.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-tb}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -rf ${2:-} > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -4 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
TPG_TUNE_DUMP=$O/tune.json timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench1.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench2.log 2>&1
echo "bench rc $?"; grep -ho '"ms_per_step": [0-9.]*' $O/bench*.log
