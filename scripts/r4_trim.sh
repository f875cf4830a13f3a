#!/bin/bash
# last-layer prefill trim: model tests, headline + batch-1 A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_tr_tests.log 2>&1 || { tail -30 gpurun_out/r4_tr_tests.log; exit 1; }
tail -1 gpurun_out/r4_tr_tests.log
hb() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --steps 6 --warmup 2 > gpurun_out/r4_tr_$tag.log 2>&1 || return $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"prefill": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_tr_$tag.log | tr '\n' ' '; echo " <- $tag"
}
hb trim DOCQA_X=1 && hb notrim DOCQA_PREFILL_TRIM=0 && hb trim2 DOCQA_X=2 && hb notrim2 DOCQA_PREFILL_TRIM=0 || exit $?
