#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for r in 1 0; do
  DOCQA_DECODE_RING=$r timeout -k 10 300 python benchmarks/bench_decode_attn.py | sed "s/^/RING=$r /" >> gpurun_out/ring.log 2>&1 || exit $?
done
