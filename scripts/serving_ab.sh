#!/bin/bash
# Same-box A/B of the online serving bench (continuous mode) under environment settings:
#   bash scripts/serving_ab.sh "A=1" "B=2" ...   (SERVE_ARGS overrides the bench arguments)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ARGS=${SERVE_ARGS:-"--rate 140 --requests 1100 --max-batch 192 --modes continuous"}
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 400 python -u benchmarks/bench_serving.py $ARGS > gpurun_out/serve_ab_$i.log 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "[$cfg] rc=$rc"; tail -5 gpurun_out/serve_ab_$i.log; exit $rc; }
  python - "$cfg" gpurun_out/serve_ab_$i.log <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith("{"):
        d = json.loads(l)
        print(f"[{sys.argv[1]}] {d['mode']} {d['value']} q/s  p50 {d['p50_latency_ms']}  p99 {d['p99_latency_ms']}  prefill_s {d['engine_prefill_s']}")
PY
done
