#!/bin/bash
# PMC passes over the grouped / per-row cascade decode probe (one counter group per run)
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc_dec
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS -d gpurun_out/pmc_dec/p1 -o run --output-format csv -- python3 scripts/group_decode_probe.py 256 > gpurun_out/pmc_dec/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc_dec/p2 -o run --output-format csv -- python3 scripts/group_decode_probe.py 256 > gpurun_out/pmc_dec/p2.log 2>&1
