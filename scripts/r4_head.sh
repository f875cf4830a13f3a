#!/bin/bash
# headline (batch 256) bench + kernel stats of a short traced run
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r4_head_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r4_head_bench.log | cut -c1-300
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/r4_prof_head -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/r4_head_prof.log 2>&1 || exit $?
mkdir -p gpurun_out/r4_prof_head && find /tmp/r4_prof_head -name '*kernel_stats.csv' -exec cp {} gpurun_out/r4_prof_head/ \;
ls gpurun_out/r4_prof_head
