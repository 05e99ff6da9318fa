# Round-2 closing measurement: headline bench (with the CPU baseline), configs 3 / 5 and the
# WGAN-GP variant, kernel-trace profile of the headline bench, per-conv trace, host overhead.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-final}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --config 3 > $O/bench_cfg3.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --gp > $O/bench_gp.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --config 5 > $O/bench_cfg5.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline > $O/prof_bench.log 2>&1
timeout -k 10 200 python -u tools/trace_step.py --no-multistream --top 90 > $O/trace_serial.log 2>&1
timeout -k 10 200 python -u tools/cpu_overhead.py > $O/cpu_overhead.log 2>&1
timeout -k 10 200 python -u tools/host_profile.py > $O/host_profile.log 2>&1
echo done
