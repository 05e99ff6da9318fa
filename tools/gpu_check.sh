# Parity suites, then a step A/B of two env settings (interleaved, 2 rounds).
#   bash tools/gpu_check.sh TAG "ENV_A=..." "ENV_B=..."
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
for rep in 1 2; do
  env $2 timeout -k 10 200 python -u bench.py --steps 15 --warmup 4 --no-cpu-baseline > $O/a$rep.log 2>&1
  env $3 timeout -k 10 200 python -u bench.py --steps 15 --warmup 4 --no-cpu-baseline > $O/b$rep.log 2>&1
done
echo done
