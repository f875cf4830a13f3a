#!/bin/bash
# Profile the headline bench on one MI355X: plain bench line first, then a rocprofv3
# kernel trace of a short run, summarised over the last timed step (trace_tail.py).
# Usage (via gpurun): bash scripts/prof_bench.sh [tag] [extra bench args...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd)
TAG=${1:-base}; shift
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ "$SKIP_BENCH" != "1" ]; then
  timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-5} --warmup 2 "$@" > gpurun_out/bench_$TAG.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "$SKIP_PROF" != "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 2 --warmup 2 "$@" > "$ROOT/gpurun_out/prof_$TAG.log" 2>&1
  rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cd "$ROOT"
  TR=$(ls gpurun_out/prof_$TAG/*kernel_trace.csv | head -1)
  WIN=${WINDOW_MS:-1300}
  python scripts/trace_tail.py "$TR" --window-ms $WIN --steps ${TAIL_STEPS:-1} --top 40 --gaps ${GAPS:-0} > gpurun_out/prof_${TAG}_tail.txt
  python scripts/phase_split.py "$TR" --last 3 > gpurun_out/prof_${TAG}_phases.txt
  rm -f gpurun_out/prof_$TAG/*kernel_trace.csv
  head -45 gpurun_out/prof_${TAG}_tail.txt; cat gpurun_out/prof_${TAG}_phases.txt
fi
exit 0
