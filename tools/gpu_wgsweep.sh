cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-sw}; mkdir -p $O
timeout -k 10 300 python3 -u tools/bench_layers.py --wg-sweep --iters 5 --only ${2:-enhance_128,add_128,conv0_res,conv5_0,enhance_64,add_64,enhance_32,enhance_16} > $O/sweep.log 2>&1
echo rc $?; cat $O/sweep.log
