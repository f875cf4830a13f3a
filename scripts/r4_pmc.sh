#!/bin/bash
# round 4: PMC passes over mgemm vs wgemm on gate|up and down (one counter group per run)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash scripts/mgemm_pmc.sh "glu 256 28672 4096 1 2" "wglu 256 28672 4096 2 1" "wglu 256 28672 4096 1 2" "mgemm 256 4096 14336 7 2" "wgemm 256 4096 14336 16 1" && for d in gpurun_out/pmc_mg/p*; do python3 scripts/pmc_summary.py $d gemm_kernel; done > gpurun_out/r4_pmc_summary.txt 2>&1; cat gpurun_out/r4_pmc_summary.txt
