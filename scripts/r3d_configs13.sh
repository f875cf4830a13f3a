#!/bin/bash
# configs 1 and 3 on the round-3 HEAD tree: ingest -> deid -> index of 1k notes, clinical-BERT NER forward
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python3 benchmarks/bench_deid.py > gpurun_out/r3d_config3_deid.log 2>&1 || exit $?
tail -3 gpurun_out/r3d_config3_deid.log
timeout -k 10 400 python3 benchmarks/bench_ingest.py > gpurun_out/r3d_config1_ingest.log 2>&1 || exit $?
tail -3 gpurun_out/r3d_config1_ingest.log
