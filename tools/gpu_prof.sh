# Kernel-trace profile of the headline bench + per-op trace (timed window summarised later).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-p}
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_bench.log 2>&1
timeout -k 10 200 python -u tools/trace_step.py --no-multistream > $O/trace.log 2>&1
echo done
