cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_group_decode_gpu.py tests/test_ivfpq_gpu.py tests/test_kernels_gpu.py -k "ivfpq or knn or group or cascade" > gpurun_out/r3_topk64_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r3_topk64_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r3_bench_persist.log 2>&1; rc=$?; tail -1 gpurun_out/r3_bench_persist.log; [ $rc -eq 0 ] || exit $rc
DOCQA_GROUP_PERSIST=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r3_bench_nopersist.log 2>&1; rc=$?; tail -1 gpurun_out/r3_bench_nopersist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/bench_ivfpq.py --data bge --n 200000 --nlist 1024 --M 64 --nq 256 > gpurun_out/r3_ivfpq_bge.log 2>&1; rc=$?; tail -8 gpurun_out/r3_ivfpq_bge.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u benchmarks/bench_serving.py --entry launch --rate 80,160 --requests 600 --modes continuous --server-log gpurun_out/r3_serve_http_srv.log > gpurun_out/r3_serve_http.log 2>&1; rc=$?; tail -3 gpurun_out/r3_serve_http.log; exit $rc
