#!/bin/bash
# IVF GPU tests; grouped decode knobs A/B on the headline (tiles per work item, ring depth)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ivfpq_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_ivf_tests.log 2>&1 || { tail -20 gpurun_out/r4_ivf_tests.log; exit 1; }
tail -1 gpurun_out/r4_ivf_tests.log
hb() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r4_gab_$tag.log 2>&1 || return $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_gab_$tag.log | tr '\n' ' '; echo " <- $tag"
}
hb t12 DOCQA_GROUP_TILES=12 && hb t24 DOCQA_GROUP_TILES=24 && hb t8 DOCQA_GROUP_TILES=8 && hb nsr4 DOCQA_GROUP_NSR=4 && hb persist DOCQA_GROUP_PERSIST=1 && hb t12b DOCQA_GROUP_TILES=12 || exit $?
