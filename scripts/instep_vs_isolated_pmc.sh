# why do isolated GEMM wins vanish inside the replayed decode step?  The
# LM head (mgemm.hip cfg 6) profiled with the same counters alone (cold weights cycled past
# the MALL) and inside bench.py's decode graph.  Effective clock = GRBM_GUI_ACTIVE / 8 /
# kernel time (MI355X_MICROARCH.md 'DVFS give-back').
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
C="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY TCC_HIT_sum TCC_MISS_sum"
timeout -s KILL 400 rocprofv3 --pmc $C --kernel-include-regex "mgemm_kernel<3, 256" -d gpurun_out/pmc_step -o step \
    -- python3 scripts/decode_step_harness.py 16 1 > gpurun_out/pmc_step.log 2>&1 || exit 1
echo ok
