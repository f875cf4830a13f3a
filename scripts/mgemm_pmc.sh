#!/bin/bash
# PMC passes over the mid-M decode GEMM probe (one counter group per run, see the gpurun rules)
# usage: bash scripts/mgemm_pmc.sh "op M N K S cfg" ...   (op: mgemm | glu | argmax | hipblaslt)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc_mg
for shape in "$@"; do
  tag=$(echo $shape | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc_mg/p1_$tag -o run --output-format csv -- python3 scripts/mgemm_pmc_probe.py $shape > gpurun_out/pmc_mg/p1_$tag.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc_mg/p2_$tag -o run --output-format csv -- python3 scripts/mgemm_pmc_probe.py $shape > gpurun_out/pmc_mg/p2_$tag.log 2>&1
done
