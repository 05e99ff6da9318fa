# hipGraph variants of the headline bench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-g}; mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph > $O/graph.log 2>&1 || echo graph failed
TPG_CONCURRENT_HINT=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph > $O/graph_nohint.log 2>&1 || echo graph_nohint failed
DEBUG_HIP_FORCE_GRAPH_QUEUES=4 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph > $O/graph_q4.log 2>&1 || echo q4 failed
TPG_MULTISTREAM=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph > $O/graph_serial.log 2>&1 || echo serial failed
TPG_MULTISTREAM=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/eager_serial.log 2>&1 || echo es failed
for f in graph graph_nohint graph_q4 graph_serial eager_serial; do echo $f $(grep -o '"ms_per_step": [0-9.]*' $O/$f.log); done
