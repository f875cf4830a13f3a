#!/bin/bash
# headline A/B: inline shared prefix in the group kernel; adaptive lead margin
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
hb() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --steps 6 --warmup 2 > gpurun_out/r4_iab_$tag.log 2>&1 || return $?
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_iab_$tag.log | tr '\n' ' '; echo " <- $tag"
}
hb base DOCQA_X=1 && hb inline DOCQA_GROUP_INLINE_PREFIX=1 && hb margin12 DOCQA_PIPELINE_LEAD_MARGIN=1.2 && hb base2 DOCQA_X=2 && hb inline2 DOCQA_GROUP_INLINE_PREFIX=1 || exit $?
