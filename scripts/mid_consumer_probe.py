"""M = 256 decode projections WITH their fused split-K consumer, per (cfg, split): the slab
bytes a split writes are read again by the consumer (QKV -> rope_cache_splitk, O / down ->
add_rmsnorm_splitk), so the GEMM alone does not rank the plans.  HIP-graph timed over
weight copies rotated past the MALL.  Usage: python scripts/mid_consumer_probe.py [M]"""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

from docqa_amd import ops
from docqa_amd.ops import reference as R

assert ops.load_native()
nat = torch.ops.docqa
M = int(sys.argv[1]) if len(sys.argv) > 1 else 256


def graph_time(fn, copies, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(copies):
            fn(i)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(copies):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * copies)


cs = R.rope_cos_sin(8192, 128, 500000.0, "cuda")
pos = torch.arange(M, device="cuda", dtype=torch.int32) + 600
slots = torch.arange(M, device="cuda", dtype=torch.int32) * 64
kc = torch.zeros(M + 1, 8, 64, 128, device="cuda", dtype=torch.bfloat16)
vc = torch.zeros_like(kc)
res = []
ONLY = os.environ.get("PROBE_ONLY", "")
for (name, N, K, plans) in [("qkv", 6144, 4096, [(2, 4), (7, 2), (7, 4), (2, 2), (2, 8)]),
                            ("o", 4096, 4096, [(7, 4), (2, 4), (7, 2), (2, 8)]),
                            ("down", 4096, 14336, [(2, 7), (2, 8), (7, 4), (2, 4), (2, 14)])]:
    if ONLY and name not in ONLY.split(","):
        continue
    nb = N * K * 2
    copies = max(2, (1 << 30) // nb + 1)
    ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(copies)]
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    gm = torch.ones(N, device="cuda", dtype=torch.bfloat16)
    for cfg, S in plans:
        if N % nat.mgemm_tile_n(cfg) or (K // 128) % S:
            continue
        gemm = graph_time(lambda i: nat.mgemm(x, ws[i], S, cfg), copies)
        if name == "qkv":
            fn = lambda i: nat.rope_cache_splitk(nat.mgemm(x, ws[i], S, cfg), pos, cs, slots, kc, vc, 32, 8, 128)
        else:
            fn = lambda i: nat.add_rmsnorm_splitk(nat.mgemm(x, ws[i], S, cfg), r, gm, 1e-5)
        both = graph_time(fn, copies)
        res.append({"proj": name, "M": M, "cfg": cfg, "S": S, "wgs": (N // nat.mgemm_tile_n(cfg)) * S,
                    "gemm_us": round(gemm, 2), "gemm_plus_consumer_us": round(both, 2)})
        print(json.dumps(res[-1]), flush=True)
    del ws
    torch.cuda.empty_cache()
