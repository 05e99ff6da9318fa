# One GPU call: parity tests, bench, trace, rocprof kernel stats.  Every GPU step has its
# own time limit and the steps are chained, so the first failure ends the call.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=${1:-run}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/$TAG/bench.log 2>&1
timeout -k 10 200 python -u tools/trace_step.py --no-multistream > gpurun_out/$TAG/trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv rocpd -d gpurun_out/$TAG/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$TAG/prof_bench.log 2>&1
echo done
