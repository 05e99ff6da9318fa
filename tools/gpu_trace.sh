# Per-conv trace of one train step (serialised local pathways) + the plain step time.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-trace}; mkdir -p $O
timeout -k 10 200 python -u tools/trace_step.py --no-multistream --top 90 > $O/trace_serial.log 2>&1
timeout -k 10 200 python -u tools/trace_step.py --top 90 > $O/trace_ms.log 2>&1
echo done
