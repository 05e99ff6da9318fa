# DP-equivalence test under env toggles (which change breaks it).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/dpab; mkdir -p $O
for ab in "TPG_GRAPH_LOSSES=0" "TPG_WGRAD_SIDE=0" "TPG_NO_RES_LINK=1" "TPG_LINEAR_FULLKERNEL=1"; do
  env $ab timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -q -k equals --timeout 290 --timeout-method thread > $O/$ab.log 2>&1 || echo "$ab failed" >> $O/summary.txt
  echo "$ab done" >> $O/summary.txt
done
echo done
