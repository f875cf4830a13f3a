#!/bin/bash
# auto tiles per item (most items within the target): batch 256 / 128 / 64
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
hb() {  # tag, batch, env...
  local tag=$1 b=$2; shift 2
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --batch $b --steps 5 --warmup 2 > gpurun_out/r4_auto2_$tag.log 2>&1 || return $?
  grep "group plan" gpurun_out/r4_auto2_$tag.log | head -1 | tr '\n' ' '
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_auto2_$tag.log | tr '\n' ' '; echo " <- $tag"
}
export DOCQA_GROUP_PLAN_LOG=1
hb b256 256 X=1 && hb b128 128 X=1 && hb b64 64 X=1 && hb b64t12 64 DOCQA_GROUP_TILES=12 && hb b256t40 256 DOCQA_GROUP_TILES=40
