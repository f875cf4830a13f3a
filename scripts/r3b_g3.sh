#!/bin/bash
# Capture-beside-busy-thread + DP share GPU tests, HTTP serving at two Poisson rates, and
# config 2 at 10M vectors with the PCA pre-rotation.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_capture_concurrency_gpu.py tests/test_dp_share_gpu.py > gpurun_out/r3b_capture_dp_tests.log 2>&1; rc=$?; tail -4 gpurun_out/r3b_capture_dp_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u benchmarks/bench_serving.py --entry launch --rate 80,160 --requests 600 --modes continuous --server-log gpurun_out/r3b_serve_http_srv.log > gpurun_out/r3b_serve_http.log; rc=$?; tail -2 gpurun_out/r3b_serve_http.log | cut -c1-900; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u benchmarks/bench_ivfpq.py --n 10000000 --nlist 4096 --M 64 --nprobe 32 > gpurun_out/r3b_ivfpq_10M_pcar.log 2>&1; rc=$?; tail -1 gpurun_out/r3b_ivfpq_10M_pcar.log | cut -c1-900; exit $rc
