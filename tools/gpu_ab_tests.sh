#!/bin/bash
# Run one pytest selection under several environments in turn (same box), e.g. an A/B of a
# library switch; a run that ends in anything but pass (0) or test failures (1) -- a fault, an
# abort, a time limit -- ends the call.
#   bash tools/gpu_ab_tests.sh <tag> "<pytest args>" "ENV=a" "ENV=b" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; ARGS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p "$O"
i=0
for e in "$@"; do
  i=$((i + 1))
  log=$(printf "%s/%02d_test.log" "$O" "$i")
  echo "== $e pytest $ARGS" | tee -a "$O/steps.txt"
  env $e timeout -k 10 900 python -u -m pytest -m gpu -q --timeout 240 --timeout-method thread $ARGS > "$log" 2>&1
  rc=$?
  echo "   rc=$rc" | tee -a "$O/steps.txt"; tail -3 "$log"
  if [[ $rc -ne 0 && $rc -ne 1 ]]; then echo "stopping (rc=$rc)"; exit $rc; fi
done
