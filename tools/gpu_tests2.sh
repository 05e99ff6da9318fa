# Full GPU suite (new round-2 tests first, so a failure there shows quickly).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-t2}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu ${3:--x} -v --timeout 400 --timeout-method thread \
  -k "${2:-}" > $O/pytest.log 2>&1
echo "pytest rc $?"
tail -5 $O/pytest.log
