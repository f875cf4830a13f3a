#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_mgemm_gpu.py tests/test_lm_head_argmax_gpu.py tests/test_wgemm_gpu.py -x -q -k "glu or argmax or packed" --timeout 120 --timeout-method thread > gpurun_out/r4_glu2_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r4_glu2_tests.log
[ $rc -ne 0 ] && exit $rc
PROBE_CFGS=1,2,17,18,20,25 timeout -k 10 300 python -u scripts/wgemm_probe.py 256 > gpurun_out/r4_glu2_probe.log 2>&1
rc=$?
cat gpurun_out/r4_glu2_probe.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/lm_head_probe.py > gpurun_out/r4_lm_head_probe.log 2>&1
rc=$?
cat gpurun_out/r4_lm_head_probe.log
exit $rc
