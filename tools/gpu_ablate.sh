# Halo-kernel timing ablations (TPG_HALO_VAR bits on the TPG_HALO_ABLATE build; wrong results).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abl}; mkdir -p $O
L=${2:-enhance_128,e128_plain,enhance_64,enhance_32,enhance_16}
for v in ${3:-0 352 864 1376 1888}; do
  echo "== var $v" >> $O/abl.log
  TPG_LIB_PATH=tp-gan_amd/ablate/libtpgan_hip.so TPG_HALO_VAR=$v timeout -k 10 100 python3 -u tools/bench_layers.py --passes fwd,dgrad --only $L >> $O/abl.log 2>&1 || exit 1
done
cat $O/abl.log
