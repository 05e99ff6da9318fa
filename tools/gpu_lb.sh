# Per-layer timings, then the default bench line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-lb}; mkdir -p $O
timeout -k 10 200 python3 -u tools/bench_layers.py ${2:-} > $O/layers.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1
echo "bench rc $?"; cat $O/layers.log; grep -o '"ms_per_step": [0-9.]*' $O/bench.log
