#!/bin/bash
# bf16 split-K slabs on the prefill split-K plans too: model GPU tests, then the reference-
# template bench (admission-size prefills) A/B 0 / 1 / 0 / 1 and the headline at the
# driver's settings.
set -o pipefail
out=gpurun_out/slab16p
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_slab16_gpu.py tests/test_models_gpu.py tests/test_pgemm_gpu.py \
  > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
i=0
for v in 0 1 0 1; do
  i=$((i + 1))
  DOCQA_SLAB_BF16=$v timeout -k 10 300 python -u bench.py --template reference --steps 5 --warmup 2 > $out/ref_${i}_$v.log 2>&1 || exit 1
  echo "ref run $i slab16=$v"
  grep '"metric"' $out/ref_${i}_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["p50_latency_ms"], d["engine_ms_per_batch"])'
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/headline.log 2>&1 || exit 1
grep '"metric"' $out/headline.log
