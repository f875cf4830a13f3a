#!/bin/bash
# Round-3 re-entry: grouped decode tests (split / deferred / persistent) then a same-box
# A/B of the deferred split plan (prefix kernel forked beside the group kernel).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_group_decode_gpu.py > gpurun_out/r3b_group_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3b_group_tests.log; [ $rc -eq 0 ] || exit $rc
BENCH_STEPS=5 bash scripts/ab_bench.sh "DOCQA_GROUP_DEFER=0" "DOCQA_GROUP_DEFER=1" "DOCQA_GROUP_DEFER=0" "DOCQA_GROUP_DEFER=1"
