#!/bin/bash
# config 5 pipeline (ingest -> deid -> embed -> kNN -> Llama-3-70B) on one GPU (TP=1), the
# round-3 kernels: batch 128 and 256, pipelined, unique questions
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for b in ${BATCHES:-256}; do
  timeout -k 10 500 python -u benchmarks/bench_pipeline.py --llm llama3-70b --batch $b --steps 3 --warmup 1 --pipelined \
    > gpurun_out/r3c_config5_70b_tp1_b$b.log 2>&1 || exit $?
  echo "b=$b: $(tail -1 gpurun_out/r3c_config5_70b_tp1_b$b.log | cut -c1-300)"
done
