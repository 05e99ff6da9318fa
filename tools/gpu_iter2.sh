# Iteration check: quick new-feature tests, full GPU parity suite, headline bench with A/B legs
# (one per ENV=VAL argument), host-overhead probe, per-conv trace.
#   bash tools/gpu_iter2.sh <tag> [ENV=VAL ...]
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-it}; mkdir -p $O
shift || true
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train.py -m gpu -x -q -k "splitk or gradlink or side_stream or folded" --timeout 150 --timeout-method thread > $O/pytest_splitk.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1
i=0
for ab in "$@"; do
  i=$((i+1))
  env $ab timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_b$i.log 2>&1
  echo "$ab" >> $O/bench_b$i.log
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench2.log 2>&1
timeout -k 10 200 python -u tools/cpu_overhead.py > $O/cpu_overhead.log 2>&1
timeout -k 10 200 python -u tools/trace_step.py --no-multistream --top 90 > $O/trace_serial.log 2>&1
echo done
