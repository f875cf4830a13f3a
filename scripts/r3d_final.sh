#!/bin/bash
# final tree re-check at round-3 HEAD (after the prep-window knob and gloo loopback binding): GPU suite + smoke + a short headline bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3d_final_gpu_suite.log 2>&1; rc=$?
tail -2 gpurun_out/r3d_final_gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3d_final_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r3d_final_smoke.log | cut -c1-120
timeout -k 10 400 python3 bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r3d_final_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3d_final_bench.log | cut -c1-300
