#!/bin/bash
# batch-1 A/B, alternating (box noise is +-5 ms between runs): XN on / off
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
b1() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --batch 1 --steps 6 --warmup 1 > gpurun_out/r4_ab_$tag.log 2>&1 || return $?
  grep -o '"p50_latency_ms": [0-9.]*\|"prefill": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_ab_$tag.log | tr '\n' ' '; echo " <- $tag"
}
b1 xn_a DOCQA_X=1 && b1 noxn_a DOCQA_DECODE_XN=0 && b1 xn_b DOCQA_X=2 && b1 noxn_b DOCQA_DECODE_XN=0 || exit $?
