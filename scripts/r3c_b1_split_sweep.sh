#!/bin/bash
# batch-1 decode attention: split count per (sequence, KV head) via the WG target
set -o pipefail
mkdir -p gpurun_out
for t in 512 8 16 32 64; do
  DOCQA_DECODE_WG_TARGET=$t timeout -k 10 300 python -u bench.py --batch 1 --steps 6 --warmup 2 > gpurun_out/b1_wg$t.log 2>&1 || exit $?
  echo "target $t: $(tail -1 gpurun_out/b1_wg$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["p50_latency_ms"], d["engine_ms_per_batch"])')"
done
