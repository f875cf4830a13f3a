#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_ivfpq_gpu.py tests/test_rag_pipelined.py > gpurun_out/r3b_bisect2.log 2>&1; echo "[ivfpq+pipelined] $(tail -1 gpurun_out/r3b_bisect2.log)"
