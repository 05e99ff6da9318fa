# Short iteration: a GPU test subset, the headline bench with A/B legs, host overhead probes.
#   bash tools/gpu_iter3.sh <tag> [ENV=VAL ...]
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-it}; mkdir -p $O
shift || true
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_train.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1
i=0
for ab in "$@"; do
  i=$((i+1))
  env $ab timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_b$i.log 2>&1
  echo "$ab" >> $O/bench_b$i.log
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench2.log 2>&1
timeout -k 10 200 python -u tools/cpu_overhead.py > $O/cpu_overhead.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo done
