#!/bin/bash
# One-GPU rehearsal of the data-parallel bench path (N ranks sharing cuda:0) and the HTTP
# serving entry; each GPU step under its own time limit, stop at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 scripts/rccl_share_probe.py > gpurun_out/r3b_rccl_share.log 2>&1; echo "rccl share probe rc=$?"; tail -4 gpurun_out/r3b_rccl_share.log
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --share-gpu --batch 64 --max-new-tokens 32 --steps 2 --warmup 1 --kv-mem-fraction 0.1 > gpurun_out/r3b_dp2_share.log 2>&1; rc=$?; echo "dp2 share rc=$rc"; tail -2 gpurun_out/r3b_dp2_share.log | cut -c1-800; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u benchmarks/bench_serving.py --entry launch --rate 80,160 --requests 600 --modes continuous --server-log gpurun_out/r3b_serve_http_srv.log > gpurun_out/r3b_serve_http.log 2>&1; rc=$?; tail -2 gpurun_out/r3b_serve_http.log | cut -c1-900; exit $rc
