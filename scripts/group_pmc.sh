#!/bin/bash
# PMC passes over the grouped-decode probe (scripts/group_decode_probe.py), one counter group per run
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc_grp
timeout -k 10 120 python3 scripts/group_decode_probe.py 256 > gpurun_out/pmc_grp/probe.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS -d gpurun_out/pmc_grp/p1 -o run --output-format csv -- python3 scripts/group_decode_probe.py 256 > gpurun_out/pmc_grp/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmc_grp/p2 -o run --output-format csv -- python3 scripts/group_decode_probe.py 256 > gpurun_out/pmc_grp/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc_grp/p3 -o run --output-format csv -- python3 scripts/group_decode_probe.py 256 > gpurun_out/pmc_grp/p3.log 2>&1
for p in p1 p2 p3; do python3 scripts/pmc_summary.py gpurun_out/pmc_grp/$p group_kernel group_split_merge flash_prefill; done > gpurun_out/pmc_grp/summary.txt 2>&1
