#!/bin/bash
# which round-4 change breaks the 4-rank shared-GPU TP test: one knob off at a time
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp DOCQA_AR_TIMEOUT_MS=3000
t() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u -m pytest tests/test_tp_gpu.py -x -q --timeout 180 --timeout-method thread -k "test-tp8" > gpurun_out/r4_tpb_$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc $(grep -o 'never arrived[^;]*' gpurun_out/r4_tpb_$tag.log | head -1) $(tail -1 gpurun_out/r4_tpb_$tag.log | cut -c1-60)"
}
t base DOCQA_X=1
t notrim DOCQA_PREFILL_TRIM=0
t noinline DOCQA_GROUP_INLINE_PREFIX=0
t nolast DOCQA_DECODE_LAST_MERGE=0
t noplans DOCQA_PREFILL_PLANS=0 DOCQA_PREFILL_MID=0
t allold DOCQA_PREFILL_TRIM=0 DOCQA_GROUP_INLINE_PREFIX=0 DOCQA_DECODE_LAST_MERGE=0 DOCQA_PREFILL_PLANS=0 DOCQA_PREFILL_MID=0
