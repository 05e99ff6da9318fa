# Same-box A/B: main library vs tp-gan_amd/ablate (per-layer fwd/dgrad timings, alternated).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ab}; mkdir -p $O
L=${2:-enhance_128,e128_plain,add_128,conv0_res,enhance_64,enhance_32,enhance_16,conv4_res,local_10}
P=${3:-fwd,dgrad}
for r in 1 2; do
  echo "== A (main) $r" >> $O/ab.log
  timeout -k 10 100 python3 -u tools/bench_layers.py --passes $P --only $L >> $O/ab.log 2>&1 || exit 1
  echo "== B (ablate) $r" >> $O/ab.log
  TPG_LIB_PATH=tp-gan_amd/ablate/libtpgan_hip.so timeout -k 10 100 python3 -u tools/bench_layers.py --passes $P --only $L >> $O/ab.log 2>&1 || exit 1
done
grep -v amdgpu.ids $O/ab.log
