#!/bin/bash
# batch-1 decode: in-kernel merges (attention partitions, projection + add + RMSNorm) tests,
# A/B bench, decode GEMM split sweep at M = 1 / 4
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "paged_decode_fused or dgemm_add_rmsnorm or add_rmsnorm_splitk" > gpurun_out/r4_b1_tests.log 2>&1 || { tail -30 gpurun_out/r4_b1_tests.log; exit 1; }
tail -1 gpurun_out/r4_b1_tests.log
b1() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --batch 1 --steps 3 --warmup 1 > gpurun_out/r4_b1_$tag.log 2>&1 || return $?
  grep -o '"p50_latency_ms": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_b1_$tag.log | tr '\n' ' '; echo " <- $tag"
}
b1 fused DOCQA_X=1 && b1 nolast DOCQA_DECODE_LAST_MERGE=0 && b1 nonorm DOCQA_DGEMM_NORM=0 && b1 neither DOCQA_DECODE_LAST_MERGE=0 DOCQA_DGEMM_NORM=0 || exit $?
timeout -k 10 300 python -u scripts/b1_probe.py 1 4 > gpurun_out/r4_b1_probe.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/pgemm_mid_probe.py 512 1024 2048 4096 > gpurun_out/r4_pgemm_mid_probe.log 2>&1 || exit $?
