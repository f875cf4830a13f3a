#!/bin/bash
# round 4: wgemm + coarse quantizer numerics, then the wgemm probe vs mgemm / hipBLASLt
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_wgemm_gpu.py tests/test_ivfpq_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_wgemm_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r4_wgemm_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/wgemm_probe.py 256 > gpurun_out/r4_wgemm_probe.log 2>&1
rc=$?
cat gpurun_out/r4_wgemm_probe.log
exit $rc
