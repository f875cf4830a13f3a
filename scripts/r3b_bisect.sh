#!/bin/bash
# Which earlier GPU test file makes test_rag_pipelined's GPU case differ (order-dependent)?
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for f in test_capture_concurrency_gpu test_group_decode_gpu test_models_gpu test_kernels_gpu test_mgemm_gpu test_pgemm_gpu test_custom_ar_gpu test_ivfpq_gpu test_kv_copy_gpu; do
  timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/$f.py tests/test_rag_pipelined.py > /tmp/b_$f.log 2>&1
  echo "[$f] $(tail -1 /tmp/b_$f.log)"
done
