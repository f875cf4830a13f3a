#!/bin/bash
# box-independent workload check: bench twice + the encoder GPU tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread -k "bert or ner or deid or embed or encoder" tests/ > gpurun_out/r4_wl_tests.log 2>&1 || { tail -30 gpurun_out/r4_wl_tests.log; exit 1; }
tail -2 gpurun_out/r4_wl_tests.log
for t in a b; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r4_wl_$t.log 2>&1 || exit $?
  tail -1 gpurun_out/r4_wl_$t.log | cut -c1-2000
done
