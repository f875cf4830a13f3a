cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r3_unique_pgemm.log 2>&1 && tail -1 gpurun_out/r3_unique_pgemm.log &&
SKIP_BENCH=1 WINDOW_MS=2600 TAIL_STEPS=2 bash scripts/prof_bench.sh r3_unique_pgemm
