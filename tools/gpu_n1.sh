# N1 (fp16 + 256x256): the new GPU tests, then a configs[4] bench line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-n1}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -rf \
  -k "f16 or 256 or config5 or golden_bf16" > $O/pytest.log 2>&1
echo "pytest rc $?"
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench5.log 2>&1
echo "bench rc $?"
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/bench5.log
