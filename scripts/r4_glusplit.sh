#!/bin/bash
# gate|up 2-way split with pipelined meet loads: tests, probe, same-box bench A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mgemm_gpu.py > gpurun_out/r4_gs_tests.log 2>&1 || { tail -30 gpurun_out/r4_gs_tests.log; exit 1; }
tail -1 gpurun_out/r4_gs_tests.log
timeout -k 10 200 python3 scripts/glu_split_probe.py > gpurun_out/r4_gs_probe.log 2>&1 || { tail -20 gpurun_out/r4_gs_probe.log; exit 1; }
grep '^{' gpurun_out/r4_gs_probe.log
hb() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r4_gs_$tag.log 2>&1 || return $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"prefill": [0-9.]*\|"decode": [0-9.]*\|"prefix_cached_frac": [0-9.]*' gpurun_out/r4_gs_$tag.log | tr '\n' ' '; echo " <- $tag"
}
hb base DOCQA_GLU_SPLIT=0 && hb split DOCQA_GLU_SPLIT=1 && hb base2 DOCQA_GLU_SPLIT=0 && hb split2 DOCQA_GLU_SPLIT=1
