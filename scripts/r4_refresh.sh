#!/bin/bash
# final tree: Mistral-7B headline, reference template (relevance / trie), batch 1
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
hb() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 400 python3 bench.py --gpus 1 "$@" > gpurun_out/r4_refresh_$tag.log 2>&1 || return $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"prefill": [0-9.]*\|"decode": [0-9.]*\|"prefix_cached_frac": [0-9.]*' gpurun_out/r4_refresh_$tag.log | tr '\n' ' '; echo " <- $tag"
}
hb mistral --llm mistral-7b --steps 5 --warmup 2 && hb ref --template reference --steps 5 --warmup 2 && \
DOCQA_CONTEXT_ORDER=trie hb reftrie --template reference --steps 5 --warmup 2 && hb b1 --batch 1 --steps 24 --warmup 4
