# Planner-knob sweep on the headline bench (env hooks read once per process).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/knobs2; mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/base.log 2>&1
for ab in "TPG_MASK_MAXPIX=16384" "TPG_CONCURRENT_HINT=0" "TPG_MULTISTREAM=0" "TPG_MASK_MAXPIX=1024"; do
  env $ab timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/$ab.log 2>&1
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/base2.log 2>&1
TPG_MASK_MAXPIX=16384 timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_train.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_mask128.log 2>&1
echo done
