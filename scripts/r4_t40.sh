#!/bin/bash
# new default (40 tiles per item): group decode GPU tests, default-args bench, lead-margin check
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_group_decode_gpu.py tests/test_models_gpu.py > gpurun_out/r4_t40_tests.log 2>&1 || { tail -30 gpurun_out/r4_t40_tests.log; exit 1; }
tail -1 gpurun_out/r4_t40_tests.log
timeout -k 10 400 python3 bench.py > gpurun_out/r4_t40_default.log 2>&1 || exit $?
tail -1 gpurun_out/r4_t40_default.log | cut -c1-260
hb() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r4_t40_$tag.log 2>&1 || return $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"prefill": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_t40_$tag.log | tr '\n' ' '; echo " <- $tag"
}
hb lead15 DOCQA_PIPELINE_LEAD_MARGIN=1.5 && hb lead10 DOCQA_PIPELINE_LEAD_MARGIN=1.0 && hb lead25 DOCQA_PIPELINE_LEAD_MARGIN=2.5 && hb lead15b DOCQA_PIPELINE_LEAD_MARGIN=1.5
