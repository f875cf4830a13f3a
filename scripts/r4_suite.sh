#!/bin/bash
# round 4: GPU suite + smoke + headline bench + batch-1 kernel trace (no library GEMM in decode)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
if [ "${SKIP_SUITE:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rA -k "not slow" > gpurun_out/r4_gpu_suite.log 2>&1; rc=$?
grep -E "passed|failed|longest peer wait" gpurun_out/r4_gpu_suite.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r4_smoke.log | cut -c1-120
fi
timeout -k 10 400 python3 bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r4_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r4_bench.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/r4_prof_b1 -o run --output-format csv -- python3 bench.py --batch 1 --steps 2 --warmup 1 > gpurun_out/r4_bench_b1.log 2>&1 || exit $?
tail -1 gpurun_out/r4_bench_b1.log | cut -c1-300
# keep only the stats summary (the full trace exceeds what gpurun copies back)
mkdir -p gpurun_out/r4_prof_b1 && find /tmp/r4_prof_b1 -name '*kernel_stats.csv' -exec cp {} gpurun_out/r4_prof_b1/ \;
ls gpurun_out/r4_prof_b1
