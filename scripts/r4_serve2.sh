#!/bin/bash
# reference-template offline bench (the service's default prompt order) + HTTP serving with
# measured token counters, offered 60 and 100 q/s
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --gpus 1 --steps 6 --warmup 2 --template reference > gpurun_out/r4_bench_reftpl.log 2>&1 || exit $?
tail -1 gpurun_out/r4_bench_reftpl.log | cut -c1-250
timeout -k 10 900 python -u benchmarks/bench_serving.py --entry launch --ignore-eos --rate 60,100 --requests 1500 --max-batch 256 --modes continuous --server-log gpurun_out/r4_serve2_srv.log > gpurun_out/r4_serve2.log; rc=$?; cut -c1-1200 gpurun_out/r4_serve2.log | tail -2; exit $rc
