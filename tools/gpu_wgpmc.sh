# HBM / L2 counters of the enhance_128 weight-gradient kernel (one pass per run).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-wg}; mkdir -p $O
P="timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv"
BL="python3 tools/bench_layers.py --iters 3"
L=${2:-enhance_128}
$P --pmc FETCH_SIZE -d $O/fetch -o run -- $BL --only $L --passes wgrad > $O/fetch.log 2>&1
$P --pmc TCC_HIT_sum TCC_MISS_sum -d $O/l2 -o run -- $BL --only $L --passes wgrad > $O/l2.log 2>&1
$P --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $O/rdreq -o run -- $BL --only $L --passes wgrad > $O/rdreq.log 2>&1
timeout -k 10 120 python3 tools/bench_layers.py > $O/layers.log 2>&1
echo done
