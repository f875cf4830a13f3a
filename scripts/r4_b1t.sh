#!/bin/bash
# batch-1 latency with the 40-tile default vs 12 (same box)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
hb() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --batch 1 --steps 24 --warmup 4 > gpurun_out/r4_b1t_$tag.log 2>&1 || return $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"prefill": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_b1t_$tag.log | tr '\n' ' '; echo " <- $tag"
}
hb t40 X=1 && hb t12 DOCQA_GROUP_TILES=12 && hb t40b X=1
