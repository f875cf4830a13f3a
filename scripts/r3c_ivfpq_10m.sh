#!/bin/bash
# config 2 at scale on the indexer path: 10M bge-base chunk embeddings -> IVF-PQ store
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1080 python -u benchmarks/bench_ivfpq.py --data bge --n 10000000 --nlist 8192 --M 96 --nprobe 64 \
  > gpurun_out/r3c_ivfpq_bge_10m.log 2> gpurun_out/r3c_ivfpq_bge_10m.err; rc=$?
tail -3 gpurun_out/r3c_ivfpq_bge_10m.err; tail -c 1500 gpurun_out/r3c_ivfpq_bge_10m.log; exit $rc
