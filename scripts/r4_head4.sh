#!/bin/bash
# final tree: headline kernel trace (stats only) + a default-args bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > gpurun_out/r4_head4_bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/r4_head4_bench_default.log | cut -c1-300
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/p4 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/r4_head4_prof.log 2>&1 || exit $?
mkdir -p gpurun_out/r4_prof_head4 && find /tmp/p4 -name "*kernel_stats.csv" -exec cp {} gpurun_out/r4_prof_head4/ \;
ls gpurun_out/r4_prof_head4
