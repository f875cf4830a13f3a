#!/bin/bash
# decode-GEMM knob sweep at 128 rows (separate processes: knobs are read once per process)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cfg in ${CFGS:-"" "DOCQA_DGEMM_XA=3"}; do
  env $cfg timeout -k 10 200 python scripts/dgemm_m128_sweep.py ${MS:-128} > gpurun_out/knob.log 2>&1 || exit 1
  echo "== $cfg"; grep '^{' gpurun_out/knob.log
done
