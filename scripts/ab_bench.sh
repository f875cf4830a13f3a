#!/bin/bash
# Same-box A/B of bench.py under environment settings (boxes differ by a few %):
#   bash scripts/ab_bench.sh "A=1" "A=0 B=2" ...   (BENCH_STEPS / BENCH_ARGS optional)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 400 python bench.py --steps ${BENCH_STEPS:-5} --warmup 2 $BENCH_ARGS > gpurun_out/ab_$i.log 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "[$cfg] rc=$rc"; tail -5 gpurun_out/ab_$i.log; exit $rc; }
  python - "$cfg" gpurun_out/ab_$i.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(f"[{sys.argv[1]}] {d['value']} q/s  p50 {d['p50_latency_ms']} ms  prefill {d['engine_ms_per_batch']['prefill']}  decode {d['engine_ms_per_batch']['decode']}")
PY
done
