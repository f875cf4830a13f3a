#!/bin/bash
# auto tiles per grouped-decode item: batch 256 (must pick 40) and smaller buckets vs fixed 40 / 12
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_group_decode_gpu.py > gpurun_out/r4_auto_tests.log 2>&1 || { tail -30 gpurun_out/r4_auto_tests.log; exit 1; }
tail -1 gpurun_out/r4_auto_tests.log
hb() {  # tag, batch, env...
  local tag=$1 b=$2; shift 2
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --batch $b --steps 5 --warmup 2 > gpurun_out/r4_auto_$tag.log 2>&1 || return $?
  grep "group plan" gpurun_out/r4_auto_$tag.log | head -1 | tr '\n' ' '
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_auto_$tag.log | tr '\n' ' '; echo " <- $tag"
}
export DOCQA_GROUP_PLAN_LOG=1
hb b256auto 256 X=1 && hb b64auto 64 X=1 && hb b64t40 64 DOCQA_GROUP_TILES=40 && hb b64t12 64 DOCQA_GROUP_TILES=12 && \
hb b128auto 128 X=1 && hb b128t40 128 DOCQA_GROUP_TILES=40 && hb b128t12 128 DOCQA_GROUP_TILES=12
