#!/bin/bash
# config 2 at scale on the indexer path with the coarse-quantizer kernel (nprobe up to 512)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1100 python -u benchmarks/bench_ivfpq.py --data bge --n 10000000 --nlist 8192 --M 96 --nprobe 128 \
  > gpurun_out/r4_ivfpq_bge_10m.log 2> gpurun_out/r4_ivfpq_bge_10m.err; rc=$?
tail -3 gpurun_out/r4_ivfpq_bge_10m.err; tail -c 1500 gpurun_out/r4_ivfpq_bge_10m.log; exit $rc
