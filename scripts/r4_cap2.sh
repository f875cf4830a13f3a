#!/bin/bash
# grouped decode: tiles per item without the plan-overflow doubling (cap 2 x bucket), same box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
hb() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r4_cap2_$tag.log 2>&1 || return $?
  grep "group plan" gpurun_out/r4_cap2_$tag.log | head -2 | tr '\n' ' '
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_cap2_$tag.log | tr '\n' ' '; echo " <- $tag"
}
export DOCQA_GROUP_PLAN_LOG=1
hb base DOCQA_GROUP_CAP_MULT=1 && hb t24 DOCQA_GROUP_CAP_MULT=2 DOCQA_GROUP_TILES=24 && hb t32 DOCQA_GROUP_CAP_MULT=2 DOCQA_GROUP_TILES=32 && \
hb t40 DOCQA_GROUP_CAP_MULT=2 DOCQA_GROUP_TILES=40 && hb t56 DOCQA_GROUP_CAP_MULT=2 DOCQA_GROUP_TILES=56 && hb t20 DOCQA_GROUP_CAP_MULT=2 DOCQA_GROUP_TILES=20 && hb base2 DOCQA_GROUP_CAP_MULT=1
