#!/bin/bash
# In-process serving (no HTTP): unique vs repeat questions at Poisson 160, max batch 128.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for qq in unique repeat; do
  timeout -k 10 400 python -u benchmarks/bench_serving.py --entry inproc --rate 160 --requests 600 --max-batch 128 --modes continuous --questions $qq > gpurun_out/r3b_serve_inproc_$qq.log 2>&1; rc=$?; tail -1 gpurun_out/r3b_serve_inproc_$qq.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc
done
