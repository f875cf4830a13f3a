#!/bin/bash
# grouped decode plan capacity: items per plan (log) and cap multiplier 1 vs 2, same box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
hb() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r4_cap_$tag.log 2>&1 || return $?
  grep "group plan" gpurun_out/r4_cap_$tag.log | sort | uniq -c | head -8
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"prefill": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_cap_$tag.log | tr '\n' ' '; echo " <- $tag"
}
hb m1 DOCQA_GROUP_PLAN_LOG=1 DOCQA_GROUP_CAP_MULT=1 && hb m2 DOCQA_GROUP_PLAN_LOG=1 DOCQA_GROUP_CAP_MULT=2 && \
hb m2t10 DOCQA_GROUP_PLAN_LOG=1 DOCQA_GROUP_CAP_MULT=2 DOCQA_GROUP_TILES=10 && hb m1b DOCQA_GROUP_CAP_MULT=1 && hb m2b DOCQA_GROUP_CAP_MULT=2
