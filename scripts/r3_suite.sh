cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pgemm_gpu.py > gpurun_out/pgemm_test2.log 2>&1; rc=$?; tail -3 gpurun_out/pgemm_test2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/pgemm_decode_probe.py 256 512 > gpurun_out/pgemm_decode_probe.log 2>&1; rc=$?; cat gpurun_out/pgemm_decode_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gpu_suite.log 2>&1; rc=$?; tail -15 gpurun_out/r3_gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r3_unique_kvfrac.log 2>&1; rc=$?; tail -1 gpurun_out/r3_unique_kvfrac.log; exit $rc
