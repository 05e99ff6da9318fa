# Quick GPU iteration: new tests + bench (graph and eager).  Steps chained; each has its own limit.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=${1:-quick}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG/bench_graph.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph > gpurun_out/$TAG/bench_eager.log 2>&1
timeout -k 10 200 python -u tools/trace_step.py --no-multistream > gpurun_out/$TAG/trace.log 2>&1
echo done
