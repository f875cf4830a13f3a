#!/bin/bash
# kNN / IVF-PQ kernel tests (block threshold top-K), config-2 recall with the PCA
# pre-rotation, then the DP rehearsal and serving runs (scripts/r3b_dp.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ivfpq_gpu.py tests/test_kernels_gpu.py -k "knn or ivfpq or topk or pool" > gpurun_out/r3b_topk_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3b_topk_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u benchmarks/bench_ivfpq.py --data bge --n 200000 --nlist 1024 --M 96 --nq 256 > gpurun_out/r3b_ivfpq_bge_pca96.log 2>&1; rc=$?; tail -1 gpurun_out/r3b_ivfpq_bge_pca96.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u benchmarks/bench_ivfpq.py --data bge --n 200000 --nlist 1024 --M 64 --nq 256 > gpurun_out/r3b_ivfpq_bge_pca64.log 2>&1; rc=$?; tail -1 gpurun_out/r3b_ivfpq_bge_pca64.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
bash scripts/r3b_dp.sh
