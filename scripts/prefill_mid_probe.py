"""Prefill projections at 513..2048 rows WITH their consumer (QKV -> RoPE + cache write,
O / down -> residual add + RMSNorm), per candidate: pgemm (256 x 256, bf16 out), gemm128,
hipBLASLt (F.linear), and the decode plans' mgemm at cfg 2 / 7 x split 1 / 2 / 4 (fp32 slabs
into the split-K consumers).  Graph-timed, weights rotated past the MALL.
Usage: python scripts/prefill_mid_probe.py [M ...]"""
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
    kc = torch.zeros((M + 63) // 64 + 1, 8, 64, 128, device="cuda", dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    for (name, N, K) in [("qkv", 6144, 4096), ("o", 4096, 4096), ("down", 4096, 14336)]:
        nb = N * K * 2
        copies = max(2, (1 << 30) // nb + 1)
        ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(copies)]
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        gm = torch.ones(N, device="cuda", dtype=torch.bfloat16)

        def plain(y):   # bf16 projection output -> consumer
            if name == "qkv":
                nat.rope_cache(y, pos, cs, slots, kc, vc, 32, 8, 128)
                return y
            return nat.add_rmsnorm(y, r, gm, 1e-5)

        def slabs(P):
            if name == "qkv":
                return nat.rope_cache_splitk(P, pos, cs, slots, kc, vc, 32, 8, 128)
            return nat.add_rmsnorm_splitk(P, r, gm, 1e-5)

        cand = {"hipblaslt": lambda i: plain(F.linear(x, ws[i])),
                "gemm128": lambda i: plain(nat.gemm(x, ws[i], None, None, 0))}
        if ops.pgemm_ok(M, N, K) or N % 256 == 0:
            cand["pgemm"] = lambda i: plain(nat.pgemm(x, ws[i], 0))
        for cfg in (2, 7):
            for S in (1, 2, 4):
                if N % nat.mgemm_tile_n(cfg) or (K // 128) % S:
                    continue
                if S == 1:
                    cand[f"m{cfg}_S1"] = (lambda i, cfg=cfg: plain(nat.mgemm(x, ws[i], 1, cfg)))
                else:
                    cand[f"m{cfg}_S{S}"] = (lambda i, cfg=cfg, S=S: slabs(nat.mgemm(x, ws[i], S, cfg)))
        out = {"M": M, "proj": name}
        for k, fn in cand.items():
            try:
                out[k] = round(graph_time(fn, copies), 1)
            except Exception as e:  # noqa: BLE001 -- a shape a candidate refuses
                out[k] = f"n/a {str(e).splitlines()[0][:40]}"
        best = min((k for k in out if k not in ("M", "proj", "hipblaslt") and isinstance(out[k], float)),
                   key=lambda k: out[k])
        out["best"], out["best_vs_lib"] = best, round(out["hipblaslt"] / out[best], 3)
        print(json.dumps(out), flush=True)
        del ws
        torch.cuda.empty_cache()
