#!/bin/bash
# full GPU suite + smoke on the current tree
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3c_gpu_suite.log 2>&1; rc=$?
tail -5 gpurun_out/r3c_gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3c_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r3c_smoke.log; exit $rc
