#!/bin/bash
# Full GPU suite on the current tree, then a rocprofv3 kernel trace of the default bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3b_gpu_suite.log 2>&1; rc=$?; tail -4 gpurun_out/r3b_gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "from __graft_entry__ import smoke; smoke()" > gpurun_out/r3b_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r3b_smoke.log; exit $rc
