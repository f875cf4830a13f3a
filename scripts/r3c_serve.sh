#!/bin/bash
# HTTP serving through services.launch, long enough for a steady-state window:
# Poisson 160 / 240 / 320 q/s x 3000 requests, max batch 256 (continuous batching)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u benchmarks/bench_serving.py --entry launch --rate ${RATES:-160,240,320} --requests ${REQS:-3000} --max-batch ${MB:-256} --modes continuous --server-log gpurun_out/r3c_serve_srv.log > gpurun_out/r3c_serve.log; rc=$?; cut -c1-700 gpurun_out/r3c_serve.log | tail -3; exit $rc
