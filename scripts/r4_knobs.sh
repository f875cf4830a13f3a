#!/bin/bash
# remaining knobs on the final tree: items target, tail-cache size (same box)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
hb() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r4_knobs_$tag.log 2>&1 || return $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"prefill": [0-9.]*\|"decode": [0-9.]*\|"prefix_cached_frac": [0-9.]*' gpurun_out/r4_knobs_$tag.log | tr '\n' ' '; echo " <- $tag"
}
hb base X=1 && hb items100 DOCQA_GROUP_ITEMS=100 && hb items170 DOCQA_GROUP_ITEMS=170 && hb tail4k DOCQA_TAIL_CACHE=4096 && hb base2 X=1
