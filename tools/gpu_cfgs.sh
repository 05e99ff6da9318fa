# Bench lines for several bench.py argument sets (same box): "args" strings.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-cf}; mkdir -p $O; shift
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 $a > $O/b$i.log 2>&1 || { echo "[$a] failed"; tail -5 $O/b$i.log; exit 1; }
  echo "[$a] $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/b$i.log | tr '\n' ' ')"
done
