# Full measurement call: parity tests, benches (configs 2 / 3 / +GP), kernel-trace profile of the
# headline bench, and the two PMC passes (FETCH_SIZE, WRITE_SIZE) of the dominant kernel.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-r2}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --identity resnet50 > $O/bench_id.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --gp > $O/bench_gp.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_bench.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $O/pmc_fetch -o run -- python3 tools/bench_layers.py --only enhance_128 --passes fwd --iters 3 > $O/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $O/pmc_write -o run -- python3 tools/bench_layers.py --only enhance_128 --passes fwd --iters 3 > $O/pmc_write.log 2>&1
echo done
