#!/bin/bash
# (1) batch-1 latency with / without TunableOp tuning of the decode-graph library GEMMs
# (2) serving admission groups at overload (Poisson 320, 2000 requests, max batch 256)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for t in 0 1; do
  DOCQA_TUNE_DECODE=$t timeout -k 10 300 python -u bench.py --batch 1 --steps 6 --warmup 2 > gpurun_out/b1_tune$t.log 2>&1 || exit $?
  echo "b1 tune=$t: $(tail -1 gpurun_out/b1_tune$t.log | cut -c1-200)"
done
export DOCQA_TUNE_DECODE=0
for cfg in "4 160" "8 80" "16 40" "2 160"; do
  set -- $cfg
  DOCQA_ADMIT_DIV=$1 DOCQA_ADMIT_WAIT_MS=$2 timeout -k 10 400 python -u benchmarks/bench_serving.py --entry launch --rate 320 \
    --requests 2000 --max-batch 256 --modes continuous > gpurun_out/r3c_admit_$1_$2.log 2>&1 || exit $?
  echo "admit div=$1 wait=$2: $(python -c "import json;d=json.loads(open('gpurun_out/r3c_admit_$1_$2.log').read().strip().splitlines()[-1]);print(d['value'],d['steady_state_qps'],d['p50_latency_ms'],d['scheduler'])")"
done
