#!/bin/bash
# retrieved-context order in the prompt: relevance (default) vs shared, same box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
hb() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r4_ord_$tag.log 2>&1 || return $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"prefill": [0-9.]*\|"decode": [0-9.]*\|"avg_prompt_tokens": [0-9.]*\|"prefix_cached_frac": [0-9.]*\|"distinct_chunks_rank0": [0-9]*' gpurun_out/r4_ord_$tag.log | tr '\n' ' '; echo " <- $tag"
}
hb rel DOCQA_CONTEXT_ORDER=relevance && hb shared DOCQA_CONTEXT_ORDER=shared && hb rel2 DOCQA_CONTEXT_ORDER=relevance && hb shared2 DOCQA_CONTEXT_ORDER=shared
