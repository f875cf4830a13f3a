cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_pgemm_gpu.py > gpurun_out/pgemm_test.log 2>&1; rc=$?; tail -15 gpurun_out/pgemm_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/pgemm_probe.py 16384 4096 1024 > gpurun_out/pgemm_probe.log 2>&1; rc=$?; cat gpurun_out/pgemm_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_custom_ar_gpu.py tests/test_tp_gpu.py > gpurun_out/tp_test.log 2>&1; rc=$?; tail -25 gpurun_out/tp_test.log; exit $rc
