#!/bin/bash
# batch-1: model/engine GPU tests (short prefill on the decode plans, QKV split 4), A/B bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py tests/test_kv_garbage_gpu.py tests/test_capture_concurrency_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_b1b_tests.log 2>&1 || { tail -30 gpurun_out/r4_b1b_tests.log; exit 1; }
tail -1 gpurun_out/r4_b1b_tests.log
b1() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --batch 1 --steps 4 --warmup 1 > gpurun_out/r4_b1b_$tag.log 2>&1 || return $?
  grep -o '"p50_latency_ms": [0-9.]*\|"prefill": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_b1b_$tag.log | tr '\n' ' '; echo " <- $tag"
}
b1 new DOCQA_X=1 && b1 noprefillmid DOCQA_PREFILL_MID=0 && b1 new2 DOCQA_X=2 || exit $?
