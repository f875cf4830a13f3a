#!/bin/bash
# grouped decode items with the inline prefix: tiles per item A/B, then a headline kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
hb() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r4_ti_$tag.log 2>&1 || return $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_ti_$tag.log | tr '\n' ' '; echo " <- $tag"
}
hb t12 DOCQA_GROUP_TILES=12 && hb t16 DOCQA_GROUP_TILES=16 && hb t10 DOCQA_GROUP_TILES=10 && hb t20 DOCQA_GROUP_TILES=20 && hb t12b DOCQA_GROUP_TILES=12 || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/p -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/r4_head3_prof.log 2>&1 || exit $?
mkdir -p gpurun_out/r4_prof_head3 && find /tmp/p -name "*kernel_stats.csv" -exec cp {} gpurun_out/r4_prof_head3/ \;
