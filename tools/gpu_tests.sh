# GPU parity tests only (one process), with a time limit.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest ${1:-tests} -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_${2:-t}.log 2>&1
