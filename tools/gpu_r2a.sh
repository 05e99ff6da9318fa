# Round-2 baseline: per-op trace, host-overhead probe, eager vs graph bench.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r2a; mkdir -p $O
timeout -k 10 200 python -u tools/trace_step.py --no-multistream > $O/trace.log 2>&1
timeout -k 10 200 python -u tools/cpu_overhead.py > $O/cpu_overhead.log 2>&1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_eager.log 2>&1
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --graph > $O/bench_graph.log 2>&1
echo done
