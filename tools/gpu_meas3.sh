# A/B: concurrency hint on / off (eager, multistream), then a trace of the default.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-m}; mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_hint.log 2>&1
TPG_CONCURRENT_HINT=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_nohint.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > $O/prof_bench.log 2>&1
for f in hint nohint; do echo $f $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$f.log); done
