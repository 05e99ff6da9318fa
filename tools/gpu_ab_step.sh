# A/B/C... of env settings on the full train step (same box, interleaved, 2 rounds).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 200 python -u bench.py --steps 15 --warmup 4 --no-cpu-baseline > $O/c${i}_r$rep.log 2>&1
  done
done
echo done
