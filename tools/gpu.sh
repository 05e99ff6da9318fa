#!/bin/bash
# The one GPU runner (replaces round 2's per-experiment tools/gpu_*.sh copies).
#
#   bash tools/gpu.sh <tag> '<step>' ['<step>' ...]
#
# Each step is one quoted string "[VAR=VAL ...] <kind> [args ...]"; the leading VAR=VAL words are
# the environment of that step only.  Steps run in order, each under its own time limit, output
# to gpurun_out/<tag>/<nn>_<kind>.log; the first failing step ends the call (no GPU work after a
# fault, abort or time limit).
#
#   test [pytest args]     GPU suite: pytest -m gpu tests (or the given files / -k expression)
#   bench [bench.py args]  headline bench (default --steps 20 --warmup 5 --no-cpu-baseline unless
#                          args are given)
#   prof [bench.py args]   rocprofv3 --kernel-trace --stats of the bench (+ tools/prof_summary.py)
#   trace [args]           tools/trace_step.py (per-conv serialised layer times)
#   layers [args]          tools/bench_layers.py
#   py <script> [args]     any python script of the repo
#   cpu                    tools/cpu_overhead.py (host enqueue time)
#   smoke                  __graft_entry__.smoke()
#   pmc <c1,c2,...> -- <python args>  one rocprofv3 --pmc pass (its own run, kill-on-timeout), e.g.
#                          'pmc SQ_WAVE_CYCLES,SQ_INSTS_MFMA -- tools/bench_layers.py --only enhance_128'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:?tag}
shift
O=gpurun_out/$TAG
mkdir -p "$O"
i=0
for spec in "$@"; do
  i=$((i + 1))
  read -r -a words <<< "$spec"
  envs=()
  while [[ ${#words[@]} -gt 0 && ${words[0]} == *=* ]]; do envs+=("${words[0]}"); words=("${words[@]:1}"); done
  kind=${words[0]}
  args=("${words[@]:1}")
  log=$(printf "%s/%02d_%s.log" "$O" "$i" "$kind")
  echo "== step $i: $spec" | tee -a "$O/steps.txt"
  case $kind in
    test)  [[ ${#args[@]} -eq 0 ]] && args=(tests)
           cmd=(timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread "${args[@]}") ;;
    bench) [[ ${#args[@]} -eq 0 ]] && args=(--steps 20 --warmup 5 --no-cpu-baseline)
           cmd=(timeout -k 10 600 python -u bench.py "${args[@]}") ;;
    prof)  [[ ${#args[@]} -eq 0 ]] && args=(--steps 10 --warmup 5 --no-cpu-baseline)
           cmd=(timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof$i" -o run -- python3 bench.py "${args[@]}") ;;
    trace) cmd=(timeout -k 10 300 python -u tools/trace_step.py "${args[@]}") ;;
    layers) cmd=(timeout -k 10 400 python -u tools/bench_layers.py "${args[@]}") ;;
    py)    cmd=(timeout -k 10 600 python -u "${args[@]}") ;;
    cpu)   cmd=(timeout -k 10 200 python -u tools/cpu_overhead.py) ;;
    smoke) cmd=(timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()") ;;
    pmc)   IFS=, read -r -a ctr <<< "${args[0]}"; rest=("${args[@]:2}")
           cmd=(timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "${ctr[@]}" -f csv -d "$O/pmc$i" -o run -- python3 "${rest[@]}") ;;
    *) echo "unknown step kind $kind"; exit 2 ;;
  esac
  env "${envs[@]}" "${cmd[@]}" > "$log" 2>&1
  rc=$?
  echo "   rc=$rc" | tee -a "$O/steps.txt"
  if [[ $kind == bench || $kind == prof ]]; then grep -o '"ms_per_step": [0-9.]*' "$log" | tee -a "$O/steps.txt"; fi
  if [[ $kind == prof && $rc -eq 0 ]]; then
    csvf=$(find "$O/prof$i" -name '*kernel_trace.csv' -print -quit)
    python tools/prof_summary.py "$csvf" --steps 10 > "$O/prof${i}_summary.txt" 2>&1 || true
  fi
  tail -3 "$log"
  if [[ $rc -ne 0 ]]; then echo "step $i failed (rc=$rc): stopping"; exit $rc; fi
done
echo done
