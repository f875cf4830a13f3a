"""LM head + greedy pick at small decode buckets: hipBLASLt + argmax kernel vs the fused
dgemm.hip EPI_ARGMAX (<= 192 rows) vs mgemm.hip cfg 6, weights rotated past the MALL.
Also the mid buckets' gate|up (fused SwiGLU) and QKV.  Usage: python scripts/lm_head_probe.py"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import torch.nn.functional as F

from benchmarks.bench_kernels import timeit
from docqa_amd import ops

ops.load_native()
nat = torch.ops.docqa
N, K = 128256, 4096
copies = 3
ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(copies)]
for M in (1, 8, 32, 64, 128, 192):
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    row = {"proj": "lm_head", "M": M}

    def t(fn):
        it = iter(range(1 << 30))
        return round(timeit(lambda: fn(ws[next(it) % copies]), iters=4 * copies), 1)

    row["hipblaslt_argmax"] = t(lambda w: nat.argmax(F.linear(x, w)))
    row["dgemm_argmax"] = t(lambda w: nat.dgemm_argmax_val(x, w, N))
    row["mgemm_argmax_c6"] = t(lambda w: nat.mgemm_argmax(x, w, N, 6))
    print(json.dumps(row), flush=True)
del ws
for name, N, K in (("gate_up", 28672, 4096), ("qkv", 6144, 4096)):
    copies = max(2, (1 << 30) // (N * K * 2) + 1)
    ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(copies)]
    for M in (64, 96, 128, 160, 192, 256):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        row = {"proj": name, "M": M}

        def t(fn):
            it = iter(range(1 << 30))
            return round(timeit(lambda: fn(ws[next(it) % copies]), iters=4 * copies), 1)

        if name == "gate_up":
            row["hipblaslt_silu"] = t(lambda w: nat.silu_mul(F.linear(x, w), True))
            if M <= 128:
                row["dgemm_glu"] = t(lambda w: nat.dgemm_glu(x, w))
            mt = (M + 255) // 256
            for c in (2, 6):
                wsb = torch.empty(mt * N * 256, device="cuda", dtype=torch.float32)
                tick = torch.zeros(2 * mt * (N // nat.mgemm_tile_n(c)) + 1, device="cuda", dtype=torch.int32)
                row[f"mgemm_glu_c{c}_S1"] = t(lambda w: nat.mgemm_glu_split(x, w, 1, c, wsb, tick))
                row[f"mgemm_glu_c{c}_S2"] = t(lambda w: nat.mgemm_glu_split(x, w, 2, c, wsb, tick))
        else:
            row["hipblaslt"] = t(lambda w: F.linear(x, w))
            for S in (2, 4, 8):
                if M <= 192:
                    row[f"dgemm_S{S}_t64"] = t(lambda w: nat.dgemm_partial(x, w, S, 64))
                row[f"mgemm_c2_S{S}"] = t(lambda w: nat.mgemm(x, w, S, 2))
                row[f"mgemm_c7_S{S}"] = t(lambda w: nat.mgemm(x, w, S, 7))
        print(json.dumps(row), flush=True)
    del ws
