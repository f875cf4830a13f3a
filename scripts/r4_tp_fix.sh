#!/bin/bash
# shared-GPU multi-rank tests with the AR workgroup cap (3 TP runs, AR and DP-share tests)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 240 python -u -m pytest tests/test_tp_gpu.py -x -q --timeout 200 --timeout-method thread -s > gpurun_out/r4_tpf_$i.log 2>&1
  echo "tp run $i rc=$? $(grep -o 'longest peer wait[^\n]*' gpurun_out/r4_tpf_$i.log | tr '\n' ' ') $(tail -1 gpurun_out/r4_tpf_$i.log | cut -c1-60)"
done
timeout -k 10 400 python -u -m pytest tests/test_custom_ar_gpu.py tests/test_dp_share_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_tpf_ar.log 2>&1; echo "ar+dp rc=$? $(tail -1 gpurun_out/r4_tpf_ar.log)"
