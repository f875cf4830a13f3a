#!/bin/bash
# Cascade decode: chunk-count sweep on a shared-prefix decode batch (gen_probe --shared),
# plus the plain path (DOCQA_CASCADE=0) for reference.  Every GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B=${B:-128}
for c in ${CHUNKS:-0 2 4 8 16}; do
  DOCQA_CASCADE_CHUNKS=$c timeout -k 10 300 python scripts/gen_probe.py --batch $B --prompt 600 --shared 448 --gen 64 --iters 2 > gpurun_out/casc_c$c.log 2>&1 || exit 1
  echo "chunks=$c $(grep 'iter 2' gpurun_out/casc_c$c.log)"
done
DOCQA_CASCADE=0 timeout -k 10 300 python scripts/gen_probe.py --batch $B --prompt 600 --shared 448 --gen 64 --iters 2 > gpurun_out/casc_off.log 2>&1 || exit 1
echo "cascade off $(grep 'iter 2' gpurun_out/casc_off.log)"
