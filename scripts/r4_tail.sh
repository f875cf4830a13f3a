#!/bin/bash
# tail-cache default 4096: full GPU suite + bench x2 + 1024 reference on the same box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not slow" > gpurun_out/r4_tail_suite.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r4_tail_suite.log | tail -1; [ $rc -eq 0 ] || { tail -40 gpurun_out/r4_tail_suite.log; exit $rc; }
hb() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r4_tail_$tag.log 2>&1 || return $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"prefill": [0-9.]*\|"decode": [0-9.]*\|"prefix_cached_frac": [0-9.]*' gpurun_out/r4_tail_$tag.log | tr '\n' ' '; echo " <- $tag"
}
hb new X=1 && hb old DOCQA_TAIL_CACHE=1024 && hb new2 X=1
