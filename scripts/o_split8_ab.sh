#!/bin/bash
# A/B: with bf16 slabs, the batch-256 O projection on 128-wide tiles at S=8 (256 workgroups,
# X re-read half as often as the 64-wide S=4 tiles; DOCQA_MID_WG_CAP=256 DOCQA_MID_NARROW=0)
# vs the default; interleaved bench.py runs on one box
set -o pipefail
out=gpurun_out/o8
mkdir -p $out
i=0
for v in 0 1 0 1; do
  i=$((i + 1))
  if [ $v = 1 ]; then e="DOCQA_MID_WG_CAP=256 DOCQA_MID_NARROW=0"; else e="DOCQA_MID_WG_CAP=224"; fi
  env $e timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $out/bench_${i}_$v.log 2>&1 || exit 1
  echo "run $i o8=$v $(grep '"metric"' $out/bench_${i}_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["p50_latency_ms"], d["engine_ms_per_batch"])')"
done
