#!/bin/bash
# serving A/B: prep collection window (embed + search batching) 0 / 4 / 8 ms at Poisson 320
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for w in 0 4 8; do
  DOCQA_PREP_WINDOW_MS=$w timeout -k 10 400 python -u benchmarks/bench_serving.py --entry launch --rate 320 \
    --requests 2500 --max-batch 256 --modes continuous > gpurun_out/r3c_prep_$w.log 2>&1 || exit $?
  echo "prep window $w ms: $(python -c "import json;d=json.loads(open('gpurun_out/r3c_prep_$w.log').read().strip().splitlines()[-1]);print(d['value'],d['steady_state_qps'],d['p50_latency_ms'],d['server_split_p50'].get('ask_batch_size_p50'),d['scheduler'])")"
done
