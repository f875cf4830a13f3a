#!/bin/bash
# reference template with relevance vs trie context order; batch-1 latency on the fixed workload
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
hb() {  # tag, args / env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --steps ${ST:-5} --warmup ${WU:-2} $ARGS > gpurun_out/r4_rb_$tag.log 2>&1 || return $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"prefill": [0-9.]*\|"decode": [0-9.]*\|"avg_prompt_tokens": [0-9.]*\|"prefix_cached_frac": [0-9.]*\|"context_order": "[a-z]*"\|"template": "[a-z_]*"' gpurun_out/r4_rb_$tag.log | tr '\n' ' '; echo " <- $tag"
}
ARGS="--template reference" hb ref_rel DOCQA_CONTEXT_ORDER=relevance && ARGS="--template reference" hb ref_trie DOCQA_CONTEXT_ORDER=trie && \
ARGS="--batch 1" ST=24 WU=4 hb b1 X=1
