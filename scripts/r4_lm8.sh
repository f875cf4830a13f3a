#!/bin/bash
# LM head on pgemm tiles (cfg 8) + context order trie: tests, probe, same-box bench A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mgemm_gpu.py -k argmax > gpurun_out/r4_lm8_tests.log 2>&1 || { tail -30 gpurun_out/r4_lm8_tests.log; exit 1; }
tail -1 gpurun_out/r4_lm8_tests.log
timeout -k 10 200 python3 scripts/lm_cfg8_probe.py > gpurun_out/r4_lm8_probe.log 2>&1 || { tail -20 gpurun_out/r4_lm8_probe.log; exit 1; }
cat gpurun_out/r4_lm8_probe.log
hb() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python3 bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/r4_lm8_$tag.log 2>&1 || return $?
  grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*\|"prefill": [0-9.]*\|"decode": [0-9.]*\|"avg_prompt_tokens": [0-9.]*\|"prefix_cached_frac": [0-9.]*' gpurun_out/r4_lm8_$tag.log | tr '\n' ' '; echo " <- $tag"
}
hb base DOCQA_LM_HEAD_CFG=6 && hb lm8 DOCQA_LM_HEAD_CFG=8 && hb lm8trie DOCQA_LM_HEAD_CFG=8 DOCQA_CONTEXT_ORDER=trie && hb base2 DOCQA_LM_HEAD_CFG=6 && hb lm8b DOCQA_LM_HEAD_CFG=8 && hb lm8trie2 DOCQA_LM_HEAD_CFG=8 DOCQA_CONTEXT_ORDER=trie
