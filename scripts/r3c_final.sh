#!/bin/bash
# round-3 final tree: GPU suite + smoke, the driver's headline command, rocprof kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3c_final_gpu_suite.log 2>&1; rc=$?
tail -3 gpurun_out/r3c_final_gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3c_final_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r3c_final_smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3c_final_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3c_final_bench.log | cut -c1-400
SKIP_BENCH=1 WINDOW_MS=1800 bash scripts/prof_bench.sh r3c_final > gpurun_out/r3c_final_prof_run.log 2>&1; rc=$?; tail -5 gpurun_out/r3c_final_prof_run.log; exit $rc
