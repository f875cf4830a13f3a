#!/bin/bash
# Round-3 re-entry: BASELINE config 2 (IVF-PQ through the indexer path, bge embeddings,
# strict + tie-aware recall) and the HTTP serving entry (services.launch).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 420 python -u benchmarks/bench_ivfpq.py --data bge --n 200000 --nlist 1024 --M ${PQ_M:-64} --nq 256 > gpurun_out/r3b_ivfpq_bge.log 2>&1; rc=$?; tail -1 gpurun_out/r3b_ivfpq_bge.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u benchmarks/bench_serving.py --entry launch --rate ${RATES:-80} --requests ${REQS:-200} --modes continuous --server-log gpurun_out/r3b_serve_http_srv.log > gpurun_out/r3b_serve_http.log 2>&1; rc=$?; tail -3 gpurun_out/r3b_serve_http.log | cut -c1-600; exit $rc
