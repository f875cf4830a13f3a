#!/bin/bash
# adaptive pipeline lead: batch-1 p50 (x2), then the headline bench + kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for t in a b; do
  timeout -k 10 300 python3 bench.py --batch 1 --steps 6 --warmup 1 > gpurun_out/r4_lead_b1_$t.log 2>&1 || exit $?
  grep -o '"p50_latency_ms": [0-9.]*\|"ms_per_step": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_lead_b1_$t.log | tr '\n' ' '; echo " <- b1 $t"
done
bash scripts/r4_head.sh
