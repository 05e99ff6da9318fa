# hipGraph parallel-branch experiment: does graph replay run the local-pathway side-stream branches concurrently?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r2b; mkdir -p $O
AMD_LOG_LEVEL=3 timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --graph > $O/log3.out 2> $O/log3.err
grep -E "max_streams|parallel streams" $O/log3.err | sort | uniq -c | head -20 > $O/graph_streams.txt || true
rm -f $O/log3.err
for q in 1 2 4 8; do
  DEBUG_HIP_FORCE_GRAPH_QUEUES=$q timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --graph > $O/bench_graph_q$q.log 2>&1 || echo "q$q failed $?"
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --graph > $O/bench_graph_nopkt.log 2>&1 || echo nopkt failed
echo done
