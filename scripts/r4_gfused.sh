#!/bin/bash
# grouped decode straight from QKV slabs: tests, then same-box A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_group_decode_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gf_tests.log 2>&1 || { tail -30 gpurun_out/r4_gf_tests.log; exit 1; }
tail -1 gpurun_out/r4_gf_tests.log
hb() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --steps 6 --warmup 2 > gpurun_out/r4_gf_$tag.log 2>&1 || return $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_gf_$tag.log | tr '\n' ' '; echo " <- $tag"
}
hb fused DOCQA_X=1 && hb unfused DOCQA_GROUP_FUSED=0 && hb fused2 DOCQA_X=2 && hb unfused2 DOCQA_GROUP_FUSED=0 || exit $?
