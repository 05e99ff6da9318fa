# A/B of the masked-dgrad map-size threshold + tuner dumps; one kernel trace (default settings).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-m}; mkdir -p $O
TPG_TUNE_DUMP=$O/tune_a.json timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_all.log 2>&1
TPG_MASK_MAXPIX=4096 TPG_TUNE_DUMP=$O/tune_b.json timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_le64.log 2>&1
TPG_MASK_MAXPIX=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_none.log 2>&1
TPG_MULTISTREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > $O/prof_bench.log 2>&1
for f in all le64 none; do echo $f $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$f.log); done
