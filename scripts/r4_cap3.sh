#!/bin/bash
# grouped decode tiles per item around 40, same box, interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
hb() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r4_cap3_$tag.log 2>&1 || return $?
  grep "group plan" gpurun_out/r4_cap3_$tag.log | head -1 | tr '\n' ' '
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_cap3_$tag.log | tr '\n' ' '; echo " <- $tag"
}
export DOCQA_GROUP_PLAN_LOG=1
hb t40 DOCQA_GROUP_TILES=40 && hb base DOCQA_GROUP_TILES=12 && hb t36 DOCQA_GROUP_TILES=36 && hb t48 DOCQA_GROUP_TILES=48 && \
hb t40b DOCQA_GROUP_TILES=40 && hb base2 DOCQA_GROUP_TILES=12 && hb t44 DOCQA_GROUP_TILES=44
