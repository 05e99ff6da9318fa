# Concurrency-share sweep (TPG_CONCURRENT_SHARE: the side-stream local-pathway ops plan for 1/share of the chip).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/share; mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/base.log 2>&1
for ab in "TPG_CONCURRENT_SHARE=2" "TPG_CONCURRENT_SHARE=3" "TPG_CONCURRENT_SHARE=6" "TPG_CONCURRENT_SHARE=8"; do
  env $ab timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/$ab.log 2>&1
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/base2.log 2>&1
echo done
