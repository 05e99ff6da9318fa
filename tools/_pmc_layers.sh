# PMC passes (one counter group per run, kernel-trace only) over the per-layer microbench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=${1:-enhance_128}
P=${2:-fwd,dgrad,wgrad}
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run -- python3 tools/bench_layers.py --only $L --passes $P --iters 3 > gpurun_out/pmc1.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run -- python3 tools/bench_layers.py --only $L --passes $P --iters 3 > gpurun_out/pmc2.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_l2 -o run -- python3 tools/bench_layers.py --only $L --passes $P --iters 3 > gpurun_out/pmc3.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES -d gpurun_out/pmc_sq -o run -- python3 tools/bench_layers.py --only $L --passes $P --iters 3 > gpurun_out/pmc4.log 2>&1
