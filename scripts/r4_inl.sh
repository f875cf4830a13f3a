#!/bin/bash
# inline-prefix default: group decode + model GPU tests, headline x2
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_group_decode_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_inl_tests.log 2>&1 || { tail -30 gpurun_out/r4_inl_tests.log; exit 1; }
tail -1 gpurun_out/r4_inl_tests.log
for t in a b; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 6 --warmup 2 > gpurun_out/r4_inl_$t.log 2>&1 || exit $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_inl_$t.log | tr '\n' ' '; echo
done
