#!/bin/bash
# grouped decode: block-table loads issued beside the context-length loads (new build) vs
# behind them (ab_lib/_docqa_C_old.so), same box, interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_group_decode_gpu.py > gpurun_out/r4_pro_tests.log 2>&1 || { tail -20 gpurun_out/r4_pro_tests.log; exit 1; }
tail -2 gpurun_out/r4_pro_tests.log
hb() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r4_pro_$tag.log 2>&1 || return $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_pro_$tag.log | tr '\n' ' '; echo " <- $tag"
}
OLD=$PWD/ab_lib/_docqa_C_old.so
hb old DOCQA_NATIVE_LIB=$OLD && hb new X=1 && hb old2 DOCQA_NATIVE_LIB=$OLD && hb new2 X=1
