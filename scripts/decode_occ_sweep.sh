#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for cfg in "4 2" "3 3" "2 4" "4 3"; do
  set -- $cfg
  DOCQA_DECODE_U=$1 DOCQA_DECODE_OCC=$2 timeout -k 10 300 python benchmarks/bench_decode_attn.py | sed "s/^/U=$1,OCC=$2 /" >> gpurun_out/occ.log 2>&1 || exit $?
done
