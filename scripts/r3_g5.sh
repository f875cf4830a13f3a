# A/B of the persistent decode's side-stream prefix fork, the overload serving run with an
# undersized KV pool (on-demand blocks + preemption), and a kernel-trace profile with the
# per-batch phase split.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
DOCQA_CASCADE_FORK=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r3_bench_persist_nofork.log 2>&1; rc=$?; tail -1 gpurun_out/r3_bench_persist_nofork.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/bench_serving.py --entry launch --rate 160 --requests 600 --modes continuous --kv-mem-fraction 0.03 --server-log gpurun_out/r3_serve_http_smallkv_srv.log > gpurun_out/r3_serve_http_smallkv.log 2>&1; rc=$?; tail -2 gpurun_out/r3_serve_http_smallkv.log; [ $rc -eq 0 ] || exit $rc
SKIP_BENCH=1 WINDOW_MS=3400 TAIL_STEPS=2 timeout -k 10 500 bash scripts/prof_bench.sh r3_final; exit $?
