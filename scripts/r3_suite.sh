cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gpu_suite.log 2>&1; rc=$?; tail -15 gpurun_out/r3_gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r3_unique_kvfrac.log 2>&1; rc=$?; tail -1 gpurun_out/r3_unique_kvfrac.log; exit $rc
