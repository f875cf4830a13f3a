"""Prefill projections at 513..2048 rows WITH their consumer (QKV -> RoPE + cache write,
O / down -> residual add + RMSNorm, gate|up -> SwiGLU), per candidate: pgemm (256 x 256,
bf16 out / fused SwiGLU), gemm128, hipBLASLt (F.linear [+ silu_mul]), the decode plans' mgemm
at cfg 2 / 7 x split 1 / 2 / 4, the 256 x 256 kernel's split-K slabs pg_S2/4/8 (fp32 slabs
into the split-K consumers: rope_cache_splitk, add_rmsnorm_splitk, silu_mul_splitk);
routed = what the forward runs (ops.prefill_route).  Llama-3-8B shapes and the Llama-3-70B TP-8 shards.  Graph-timed,
weights rotated past the MALL.
Usage: python scripts/prefill_mid_probe.py [M ...]   (PROBE_PROJ=qkv,70b_down,... filters)"""
import os
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import torch.nn.functional as F

from docqa_amd import ops
from docqa_amd.ops import reference as R

assert ops.load_native()
nat = torch.ops.docqa


def graph_time(fn, copies, reps=10):
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


Ms = [int(a) for a in sys.argv[1:]] or [768, 1024, 1536, 2048]
cs = R.rope_cos_sin(8192, 128, 500000.0, "cuda")
for M in Ms:
    pos = torch.arange(M, device="cuda", dtype=torch.int32) % 4000
    slots = torch.arange(M, device="cuda", dtype=torch.int32)
    kc = torch.zeros((M + 63) // 64 + 1, 8, 64, 128, device="cuda", dtype=torch.bfloat16)   # [blocks, Hkv, 64, D]
    vc = torch.zeros_like(kc)
    only = os.environ.get("PROBE_PROJ", "")
    for (name, N, K, heads) in [("qkv", 6144, 4096, (32, 8)), ("o", 4096, 4096, None), ("down", 4096, 14336, None),
                                ("gate_up", 28672, 4096, "glu"), ("70b_qkv", 1280, 8192, (8, 1)),
                                ("70b_o", 8192, 1024, None), ("70b_gate_up", 7168, 8192, "glu"),
                                ("70b_down", 8192, 3584, None)]:
        if only and name not in only.split(","):
            continue
        glu = heads == "glu"
        nb = N * K * 2
        copies = max(2, (1 << 30) // nb + 1)
        ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(copies)]
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)

        if not glu:
            r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
            gm = torch.ones(N, device="cuda", dtype=torch.bfloat16)

        def plain(y):   # bf16 projection output -> consumer
            if glu:
                return ops.silu_mul(y, interleaved=True)
            if isinstance(heads, tuple):
                nat.rope_cache(y, pos, cs, slots, kc, vc, heads[0], heads[1], 128)
                return y
            return nat.add_rmsnorm(y, r, gm, 1e-5)

        def slabs(P):
            if glu:
                return nat.silu_mul_splitk(P)
            if isinstance(heads, tuple):
                return nat.rope_cache_splitk(P, pos, cs, slots, kc, vc, heads[0], heads[1], 128)
            return nat.add_rmsnorm_splitk(P, r, gm, 1e-5)

        cand = {"hipblaslt": lambda i: plain(F.linear(x, ws[i]))}
        route, rfn = ops.prefill_route(M, N, K, glu=glu, down=name.endswith("down"))

        def routed(i):   # what the prefill forward runs (ops.prefill_route) + its consumer
            y = rfn(x, ws[i])
            if glu:
                return y
            return slabs(y) if y.dim() == 3 else plain(y)

        cand["routed"] = routed
        if glu:
            cand["gemm128"] = lambda i: nat.gemm(x, ws[i], None, None, 4)
            cand["pgemm"] = lambda i: nat.pgemm(x, ws[i], 1)
        else:
            cand["gemm128"] = lambda i: plain(nat.gemm(x, ws[i], None, None, 0))
            if N % 256 == 0:
                cand["pgemm"] = lambda i: plain(nat.pgemm(x, ws[i], 0))
        if N % 256 == 0:
            for S in (2, 4, 8):
                if K % (S * 128) == 0 and ((M + 255) // 256) * (N // 256) * S <= 512:
                    cand[f"pg_S{S}"] = (lambda i, S=S: slabs(nat.pgemm_partial(x, ws[i], S)))
        for cfg in (() if glu else (2, 7)):
            for S in (1, 2, 4):
                if N % nat.mgemm_tile_n(cfg) or (K // 128) % S:
                    continue
                if S == 1:
                    cand[f"m{cfg}_S1"] = (lambda i, cfg=cfg: plain(nat.mgemm(x, ws[i], 1, cfg)))
                else:
                    cand[f"m{cfg}_S{S}"] = (lambda i, cfg=cfg, S=S: slabs(nat.mgemm(x, ws[i], S, cfg)))
        out = {"M": M, "proj": name, "route": route}
        for k, fn in cand.items():
            try:
                out[k] = round(graph_time(fn, copies), 1)
            except Exception as e:  # noqa: BLE001 -- a shape a candidate refuses
                out[k] = f"n/a {str(e).splitlines()[0][:40]}"
        best = min((k for k in out if k not in ("M", "proj", "route", "hipblaslt", "routed")
                    and isinstance(out[k], float)), key=lambda k: out[k])
        out["best"], out["best_vs_lib"] = best, round(out["hipblaslt"] / out[best], 3)
        out["routed_vs_lib"] = round(out["hipblaslt"] / out["routed"], 3)
        print(json.dumps(out), flush=True)
        del ws
        torch.cuda.empty_cache()
