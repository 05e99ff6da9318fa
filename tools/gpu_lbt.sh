# GPU op tests (conv parity), per-layer timings, the default bench line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-lbt}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/bench_layers.py ${2:-} > $O/layers.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
echo "bench rc $?"; cat $O/layers.log; grep -o '"ms_per_step": [0-9.]*' $O/bench.log
