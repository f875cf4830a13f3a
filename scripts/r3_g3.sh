# Config-5 functional rehearsal on ONE GPU: Llama-3-70B TP=8 (8 ranks share the card,
# gloo for host collectives, the IPC all-reduce forced on), full ingest -> deid -> embed ->
# sharded kNN -> generate pipeline.  Throughput is meaningless (8 ranks time-share one
# GPU); this proves the 8-rank fused path runs end to end with the real 70B shapes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 benchmarks/bench_pipeline.py --llm llama3-70b --share-gpu --batch 16 --steps 1 --warmup 1 --max-new-tokens 32 --notes 200 > gpurun_out/r3_config5_70b_tp8_sharegpu.log 2>&1; rc=$?; tail -5 gpurun_out/r3_config5_70b_tp8_sharegpu.log; exit $rc
