# Iteration check: full GPU parity suite, headline bench (A/B against an env hook), per-conv trace.
#   bash tools/gpu_iter2.sh <tag> [ENV=VAL for the B leg]
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-it}; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q -k "splitk or gradlink" --timeout 100 --timeout-method thread > $O/pytest_splitk.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1
if [ -n "$2" ]; then env $2 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_b.log 2>&1; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench2.log 2>&1
timeout -k 10 200 python -u tools/trace_step.py --no-multistream --top 90 > $O/trace_serial.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph > $O/bench_graph.log 2>&1
echo done
