#!/bin/bash
# Same-box A/B of the service's GIL switch interval under HTTP Poisson load.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for sw in ${SWITCHES:-5 0.5}; do
  DOCQA_GIL_SWITCH_MS=$sw timeout -k 10 500 python -u benchmarks/bench_serving.py --entry launch --rate ${RATES:-80,160} --requests 600 --max-batch 128 --modes continuous --server-log gpurun_out/r3b_serve_sw${sw}_srv.log > gpurun_out/r3b_serve_sw$sw.log; rc=$?
  python3 - "$sw" gpurun_out/r3b_serve_sw$sw.log <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith("{"):
        d = json.loads(l)
        print(f"[switch {sys.argv[1]} ms] rate {d['offered_rate']}: {d['value']} q/s p50 {d['p50_latency_ms']} p90 {d['p90_latency_ms']} steps {d['scheduler']['steps']}")
PY
  [ $rc -eq 0 ] || exit $rc
done
