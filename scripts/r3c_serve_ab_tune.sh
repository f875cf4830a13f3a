#!/bin/bash
# serving A/B: TunableOp tuning of the decode-graph GEMMs at capture (default) vs off
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for t in 0 1; do
  DOCQA_TUNE_DECODE=$t timeout -k 10 500 python -u benchmarks/bench_serving.py --entry launch --rate 320 --requests 2000 \
    --max-batch 256 --modes continuous --server-log gpurun_out/r3c_serve_tune${t}_srv.log > gpurun_out/r3c_serve_tune$t.log 2>&1 || exit $?
  echo "tune=$t: $(cut -c1-330 gpurun_out/r3c_serve_tune$t.log | tail -1)"
done
