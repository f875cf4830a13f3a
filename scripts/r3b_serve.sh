#!/bin/bash
# HTTP serving through services.launch at Poisson 80 / 160 / 240 q/s (continuous batching).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u benchmarks/bench_serving.py --entry launch --rate ${RATES:-80,160,240} --requests ${REQS:-600} --max-batch ${MB:-128} --modes continuous --server-log gpurun_out/r3b_serve_http_srv.log > gpurun_out/r3b_serve_http.log; rc=$?; cut -c1-600 gpurun_out/r3b_serve_http.log | tail -3; exit $rc
