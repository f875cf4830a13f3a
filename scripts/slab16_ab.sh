#!/bin/bash
# A/B of the bf16 split-K slabs (DOCQA_SLAB_BF16) on the batch-256 headline: GPU tests of the
# kernels first, then interleaved bench.py runs (0 / 1 / 0 / 1) on one box.
set -o pipefail
out=gpurun_out/slab16
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_slab16_gpu.py tests/test_mgemm_gpu.py "tests/test_models_gpu.py::test_llama_mid_batch_decode_native_vs_reference" \
  > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -3 $out/tests.log
i=0
for v in 0 1 0 1; do
  i=$((i + 1))
  DOCQA_SLAB_BF16=$v timeout -k 10 300 python -u bench.py --steps ${STEPS:-10} --warmup 3 > $out/bench_${i}_$v.log 2>&1 || exit 1
  echo "run $i slab16=$v"
  grep '"metric"' $out/bench_${i}_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["p50_latency_ms"], d["engine_ms_per_batch"])'
done
