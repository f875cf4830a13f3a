#!/bin/bash
# sweep decode-attention knobs on HBM-resident caches (one process per setting)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for u in ${SWEEP_U:-2}; do
  for t in ${SWEEP_TARGETS:-512}; do
    DOCQA_DECODE_U=$u DOCQA_DECODE_WG_TARGET=$t timeout -k 10 300 python benchmarks/bench_decode_attn.py >> gpurun_out/decode_sweep.log 2>&1 || exit $?
  done
done
