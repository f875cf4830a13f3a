#!/bin/bash
# BASELINE config 5 rehearsal on the one-GPU box: Llama-3-70B TP=8 (eight ranks sharing the
# GPU, gloo process group, the IPC all-reduce with fused residual + RMSNorm between the
# ranks' processes), index sharded x8.  Correctness of the TP=8 path, not speed.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 benchmarks/bench_pipeline.py --llm llama3-70b --share-gpu --batch ${B:-8} --steps 1 --warmup 1 --max-new-tokens ${T:-16} --notes 100 > gpurun_out/r3b_config5_70b_tp8_share.log 2>&1; rc=$?; tail -3 gpurun_out/r3b_config5_70b_tp8_share.log | cut -c1-1500; exit $rc
