# wgrad tile / split sweep (tuning data for the planner's cost model)
out=${1:-gpurun_out/sw.log}
for cfg in 256,128 128,128 128,64 64,64; do
  for ks in 1 2 4 8 16 32; do
    echo "== $cfg ks $ks" >> $out
    TPG_WGRAD_FORCE=$cfg,$ks timeout -k 10 60 python3 tools/bench_layers.py --passes wgrad --iters 5 \
      --only enhance_128,add_128,conv0_res,enhance_64,add_64,enhance_32,enhance_16,conv4_res,local_10,local_20 >> $out 2>&1 || exit 1
  done
done
