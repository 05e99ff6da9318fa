# wgrad tile / split sweep (tuning data for the planner's cost model)
for cfg in 256,128 128,128 128,64 64,128 64,64; do
  for ks in 1 2 4 8 16 32 64; do
    echo "== $cfg ks $ks" >> gpurun_out/sw3.log
    TPG_WGRAD_FORCE=$cfg,$ks timeout -k 10 60 python3 tools/bench_layers.py --passes wgrad --iters 5 \
      --only enhance_128,add_128,enhance_64,enhance_16,conv4_res,local_10 >> gpurun_out/sw3.log 2>&1 || exit 1
  done
done
