#!/bin/bash
# late round-6 verification on one box: full GPU suite, smoke(), HTTP serving at offered 60 /
# 100 q/s (reference prompt, --ignore-eos), the headline at the driver's settings with
# DOCQA_SLAB_BF16 0 then 1 (same box)
set -o pipefail
out=gpurun_out/late
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $out/suite.log 2>&1 || { tail -30 $out/suite.log; exit 1; }
tail -1 $out/suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 420 python -u benchmarks/bench_serving.py --rate 60,100 --requests 1500 --max-batch 256 \
  --ignore-eos --modes continuous --server-log $out/srv.log > $out/serve.log 2>&1 || { tail -20 $out/serve.log; exit 1; }
grep -h '^{' $out/serve.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    if 'offered_rate' in d:
        print('serving', d['offered_rate'], d['value'], d['p50_latency_ms'], d['p90_latency_ms'])"
for v in 0 1; do
  DOCQA_SLAB_BF16=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/head_$v.log 2>&1 || exit 1
  echo "headline slab16=$v $(grep '"metric"' $out/head_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["p50_latency_ms"], d["engine_ms_per_batch"])')"
done
