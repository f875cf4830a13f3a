#!/bin/bash
# with 40-tile items: ring depth 4 (2 workgroups / CU) and the inline prefix re-checked, same box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
hb() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r4_t40b_$tag.log 2>&1 || return $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"prefill": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_t40b_$tag.log | tr '\n' ' '; echo " <- $tag"
}
hb base X=1 && hb nsr4 DOCQA_GROUP_NSR=4 && hb noinline DOCQA_GROUP_INLINE_PREFIX=0 && hb nsr4t64 DOCQA_GROUP_NSR=4 DOCQA_GROUP_TILES=64 && hb base2 X=1 && hb nsr4b DOCQA_GROUP_NSR=4
