# SQ counter pass (one group) over one layer's kernels: MFMA / LDS / wait breakdown.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=${1:-enhance_128}; P=${2:-fwd}; T=${3:-sq}
mkdir -p gpurun_out/$T
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS -f csv -d gpurun_out/$T/a -o run -- python3 tools/bench_layers.py --only $L --passes $P --iters 3 > gpurun_out/$T/a.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d gpurun_out/$T/b -o run -- python3 tools/bench_layers.py --only $L --passes $P --iters 3 > gpurun_out/$T/b.log 2>&1
echo done
