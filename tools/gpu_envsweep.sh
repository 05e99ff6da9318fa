# Bench line per environment setting (same box): "NAME=VAL,NAME2=VAL ..." arguments.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-es}; mkdir -p $O; shift
for cfg in "$@"; do
  envs=$(echo "$cfg" | tr ',' ' ')
  [ "$cfg" = "default" ] && envs=""
  env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 > $O/b.log 2>&1 || { echo "$cfg failed"; tail -3 $O/b.log; exit 1; }
  echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' $O/b.log)"
done
