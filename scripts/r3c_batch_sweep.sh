#!/bin/bash
# headline batch size vs p50: unique questions, default stack, batch 224 / 240 / 256
set -o pipefail
mkdir -p gpurun_out
for b in 224 240 256; do
  timeout -k 10 300 python -u bench.py --batch $b --steps 6 --warmup 2 > gpurun_out/bench_b$b.log 2>&1 || exit $?
done
