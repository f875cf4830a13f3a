#!/bin/bash
# GPU suite + smoke + headline bench x2 (workload must be identical across runs and boxes)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not slow" > gpurun_out/r4_final_suite.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r4_final_suite.log | tail -3; [ $rc -eq 0 ] || { tail -40 gpurun_out/r4_final_suite.log; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_final_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r4_final_smoke.log | cut -c1-120
for t in a b; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps ${STEPS:-5} --warmup ${WARM:-2} > gpurun_out/r4_final_bench_$t.log 2>&1 || exit $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"prefill": [0-9.]*\|"decode": [0-9.]*\|"avg_prompt_tokens": [0-9.]*\|"prefix_cached_frac": [0-9.]*\|"distinct_chunks_rank0": [0-9]*\|"context_order": "[a-z]*"' gpurun_out/r4_final_bench_$t.log | tr '\n' ' '; echo " <- $t"
done
