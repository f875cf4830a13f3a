#!/bin/bash
# prefill mid-M plans: model tests, batch-4 bench A/B, HTTP serving A/B at 60 q/s
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_pp_tests.log 2>&1 || { tail -30 gpurun_out/r4_pp_tests.log; exit 1; }
tail -1 gpurun_out/r4_pp_tests.log
b4() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --batch 4 --steps 4 --warmup 1 > gpurun_out/r4_pp_b4_$tag.log 2>&1 || return $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"prefill": [0-9.]*\|"decode": [0-9.]*' gpurun_out/r4_pp_b4_$tag.log | tr '\n' ' '; echo " <- b4 $tag"
}
b4 plans DOCQA_X=1 && b4 noplans DOCQA_PREFILL_PLANS=0 || exit $?
sv() {
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u benchmarks/bench_serving.py --entry launch --ignore-eos --rate 60 --requests 1200 --max-batch 256 --modes continuous --server-log gpurun_out/r4_pp_srv_$tag.log > gpurun_out/r4_pp_serve_$tag.log || return $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"p90_latency_ms": [0-9.]*' gpurun_out/r4_pp_serve_$tag.log | tr '\n' ' '; echo " <- serve $tag"
}
sv plans DOCQA_X=1 && sv noplans DOCQA_PREFILL_PLANS=0 || exit $?
