#!/bin/bash
# A/B of the split bf16-slab gate|up (DOCQA_GLU_SPLIT16) on the batch-256 headline: GPU tests
# first, then interleaved bench.py runs (0 / 1 / 0 / 1) on one box, then a kernel-stats run.
set -o pipefail
out=gpurun_out/glu16
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_slab16_gpu.py "tests/test_models_gpu.py::test_llama_mid_batch_decode_native_vs_reference" \
  > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
i=0
for v in 0 1 0 1; do
  i=$((i + 1))
  DOCQA_GLU_SPLIT16=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $out/bench_${i}_$v.log 2>&1 || exit 1
  echo "run $i glu16=$v $(grep '"metric"' $out/bench_${i}_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["p50_latency_ms"], d["engine_ms_per_batch"])')"
done
