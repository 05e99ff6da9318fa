# Kernel trace of the headline bench with the local pathways serialised (per-layer attribution by grid).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r2c; mkdir -p $O
TPG_MULTISTREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > $O/prof_bench.log 2>&1
echo done
