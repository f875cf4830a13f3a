#!/bin/bash
# The one gpurun driver (replaces the per-experiment r*_*.sh wrappers of rounds 1-4).
#
#   gpurun --timeout 1200 -- 'bash scripts/gpu.sh STEP [STEP ...]'
#
# Steps run in order, each under its own `timeout -k 10`, output in gpurun_out/<n>_<kind>.log;
# the first failing step ends the call (no retries: a fault, abort or time limit must be read,
# not repeated).  STEP forms (the argument text after the first ':' is split by the shell):
#   suite[:<pytest args>]           python -m pytest tests -m gpu (timeout 900 s)
#   smoke                           __graft_entry__.smoke()
#   bench[:<bench.py args>]         python bench.py ... ; the JSON line is echoed
#   py:<script> [args]              any python script (probes, micro-benchmarks; 600 s)
#   prof:<tag>:<script> [args]      rocprofv3 --kernel-trace --stats -> gpurun_out/prof_<tag>/
#   env:NAME=VALUE                  export NAME for the steps after it (A/B knobs)
#   pmc:<tag>:<counters>:<script> [args]
#                                   rocprofv3 --pmc <counters> --kernel-trace --stats (one pass;
#                                   counters space-separated inside the step, keep within the
#                                   per-block slot limits) -> gpurun_out/pmc_<tag>/
# Env: STEP_TIMEOUT overrides the per-step limit (seconds).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
n=0
for step in "$@"; do
  n=$((n + 1))
  kind="${step%%:*}"
  arg=""
  [ "$kind" != "$step" ] && arg="${step#*:}"
  log="gpurun_out/${n}_${kind}.log"
  t0=$(date +%s)
  case "$kind" in
    env)
      export "$arg"; echo "[gpu.sh] export $arg"; continue ;;
    suite)
      timeout -k 10 "${STEP_TIMEOUT:-900}" python -u -m pytest tests -m gpu -x -q --timeout 300 \
        --timeout-method thread $arg > "$log" 2>&1 ;;
    smoke)
      timeout -k 10 "${STEP_TIMEOUT:-600}" python -c "from __graft_entry__ import smoke; smoke()" > "$log" 2>&1 ;;
    bench)
      timeout -k 10 "${STEP_TIMEOUT:-900}" python bench.py $arg > "$log" 2>&1 ;;
    py)
      timeout -k 10 "${STEP_TIMEOUT:-600}" python -u $arg > "$log" 2>&1 ;;
    prof)
      tag="${arg%%:*}"; read -r script rest <<< "${arg#*:}"
      out="$ROOT/gpurun_out/prof_$tag"
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 "${STEP_TIMEOUT:-600}" rocprofv3 --kernel-trace --stats \
        -d "$out" -o run --output-format csv -- python3 "$ROOT/$script" $rest) > "$log" 2>&1
      rc=$?
      rm -f "$out"/*/*kernel_trace.csv "$out"/*kernel_trace.csv 2>/dev/null
      ( exit $rc ) ;;
    pmc)
      tag="${arg%%:*}"; r2="${arg#*:}"; ctrs="${r2%%:*}"; read -r script rest <<< "${r2#*:}"
      out="$ROOT/gpurun_out/pmc_$tag"
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL "${STEP_TIMEOUT:-300}" rocprofv3 --pmc $ctrs --kernel-trace \
        --stats -d "$out" -o run --output-format csv -- python3 "$ROOT/$script" $rest) > "$log" 2>&1 ;;
    *)
      echo "unknown step '$step'"; exit 2 ;;
  esac
  rc=$?
  echo "[gpu.sh] step $n ($kind) rc=$rc in $(( $(date +%s) - t0 )) s -> $log"
  tail -3 "$log"
  if [ $rc -ne 0 ]; then
    tail -40 "$log"
    exit $rc
  fi
done
exit 0
