#!/bin/bash
# round-3 extras: the reference's own generator (Mistral-7B v0.3 shapes) on the headline
# workload, and the single-question latency (batch 1) of the default Llama-3-8B stack
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --llm mistral-7b --steps 5 --warmup 2 > gpurun_out/bench_mistral.log 2>&1 &&
timeout -k 10 400 python -u bench.py --batch 1 --steps 8 --warmup 2 > gpurun_out/bench_b1.log 2>&1
