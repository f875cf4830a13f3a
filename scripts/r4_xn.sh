#!/bin/bash
# batch-1 XN (in-kernel residual add + RMSNorm input rows): tests, A/B bench, batch-1 kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "xn or decode or dgemm or llama or embed or argmax" > gpurun_out/r4_xn_tests.log 2>&1 || { tail -40 gpurun_out/r4_xn_tests.log; exit 1; }
tail -1 gpurun_out/r4_xn_tests.log
b1() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --batch 1 --steps 4 --warmup 1 > gpurun_out/r4_xn_$tag.log 2>&1 || return $?
  grep -o '"p50_latency_ms": [0-9.]*\|"prefill": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_xn_$tag.log | tr '\n' ' '; echo " <- $tag"
}
b1 xn DOCQA_X=1 && b1 noxn DOCQA_DECODE_XN=0 && b1 xn2 DOCQA_X=2 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/r4_prof_xn -o run --output-format csv -- python3 bench.py --batch 1 --steps 2 --warmup 1 > gpurun_out/r4_xn_prof.log 2>&1 || exit $?
mkdir -p gpurun_out/r4_prof_xn && find /tmp/r4_prof_xn -name '*kernel_stats.csv' -exec cp {} gpurun_out/r4_prof_xn/ \;
