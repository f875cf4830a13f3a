#!/bin/bash
# round 4: the 4-rank shared-GPU TP test with one hardware queue per process (4 queues in
# all) -- does rank 0 still "never arrive"?  and the 8-rank DP share-GPU bench likewise
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
GPU_MAX_HW_QUEUES=1 DOCQA_AR_TIMEOUT_MS=30000 timeout -k 10 400 python -u -m pytest tests/test_tp_gpu.py tests/test_custom_ar_gpu.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r4_hwq1_tp.log 2>&1; rc=$?
grep -E "passed|failed|longest peer wait|never arrived" gpurun_out/r4_hwq1_tp.log | tail -8
[ $rc -eq 0 ] || exit $rc
GPU_MAX_HW_QUEUES=1 DOCQA_AR_TIMEOUT_MS=30000 timeout -k 10 600 python -u -m pytest tests/test_dp_share_gpu.py -x -q -s --timeout 500 --timeout-method thread > gpurun_out/r4_hwq1_dp.log 2>&1; rc=$?
grep -E "passed|failed|never arrived|Error" gpurun_out/r4_hwq1_dp.log | tail -8
exit $rc
