#!/bin/bash
# HTTP serving through services.launch with every answer decoding max_new_tokens
# (--ignore-eos: no early-EOS completions), offered 100 q/s (below saturation) and 160 q/s,
# plus the deid service path with NER in the loop vs the engine alone
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u benchmarks/bench_deid_service.py --docs 2048 --batch-docs 64 > gpurun_out/r4_deid_service.log 2> gpurun_out/r4_deid_service.err || { tail -5 gpurun_out/r4_deid_service.err; exit 1; }
tail -1 gpurun_out/r4_deid_service.log | cut -c1-400
timeout -k 10 900 python -u benchmarks/bench_serving.py --entry launch --ignore-eos --rate ${RATES:-100,160} --requests ${REQS:-2000} --max-batch ${MB:-256} --modes continuous --server-log gpurun_out/r4_serve_srv.log > gpurun_out/r4_serve.log; rc=$?; cut -c1-900 gpurun_out/r4_serve.log | tail -3; exit $rc
