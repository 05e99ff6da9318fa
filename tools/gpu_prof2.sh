# Default bench line (no CPU baseline) and a kernel trace of the same step.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-p}; mkdir -p $O
TPG_TUNE_DUMP=$O/tune.json timeout -k 10 300 python -u bench.py --no-cpu-baseline ${2:-} > $O/bench.log 2>&1
grep -o '"ms_per_step": [0-9.]*' $O/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline ${2:-} > $O/prof_bench.log 2>&1
echo done
