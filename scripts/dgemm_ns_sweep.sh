#!/bin/bash
# ring-depth sweep of the split-K decode projection (one process per setting)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for ns in ${SWEEP_NS:-4 6 8}; do
  echo "NS=$ns" >> gpurun_out/ns_sweep.log
  DOCQA_DGEMM_NS=$ns timeout -k 10 300 python scripts/dgemm_partial_sweep.py 64 >> gpurun_out/ns_sweep.log 2>&1 || exit $?
done
