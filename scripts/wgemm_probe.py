"""wgemm.hip (weights in VGPRs) vs mgemm.hip (both operands through LDS) vs hipBLASLt on
the Llama-3-8B decode projections at M rows, weights rotated past the 256 MB MALL.
Usage: python scripts/wgemm_probe.py [M ...]   (PROBE_CFGS=1,2,3,4,9,... to pick variants)"""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import torch.nn.functional as F

from benchmarks.bench_kernels import timeit
from docqa_amd import ops

ops.load_native()
nat = torch.ops.docqa
Ms = [int(a) for a in sys.argv[1:]] or [256]
CFGS = [int(c) for c in os.environ.get("PROBE_CFGS", "1,2,3,4,9,10,11,12").split(",")]
for (name, N, K) in [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096),
                     ("down", 4096, 14336), ("lm_head", 128256, 4096)]:
    nb = N * K * 2
    copies = max(2, (1 << 30) // nb + 1)
    ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(copies)]
    for M in Ms:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        row = {"proj": name, "M": M, "weights_MB": round(nb / 2 ** 20, 1)}

        def t(fn):
            it = iter(range(1 << 30))
            return round(timeit(lambda: fn(ws[next(it) % copies]), iters=4 * copies), 1)

        row["hipblaslt"] = t(lambda w: F.linear(x, w))
        if name == "gate_up":
            row["mgemm_glu_c2"] = t(lambda w: nat.mgemm_glu(x, w, 2))
            mt = (M + 255) // 256
            for c in (3, 5, 6):
                wsb = torch.empty(mt * N * 256, device="cuda", dtype=torch.float32)
                tick = torch.zeros(2 * mt * (N // nat.mgemm_tile_n(c)) + 1, device="cuda", dtype=torch.int32)
                row[f"mgemm_glu_c{c}_S2"] = t(lambda w: nat.mgemm_glu_split(x, w, 2, c, wsb, tick))
        elif name == "lm_head":
            row["mgemm_argmax_c6"] = t(lambda w: nat.mgemm_argmax(x, w, N, 6))
        else:
            S, c = ops.mid_plan(M, N, K)
            if S:
                row[f"mgemm_c{c}_S{S}"] = t(lambda w: nat.mgemm(x, w, S, c))
        wsp = None
        for cfg in CFGS:
            if cfg >= 16 and wsp is None:     # fragment-major packed copies of the rotation
                wsp = [ops.pack_fragments(w) for w in ws]
            wl = wsp if cfg >= 16 else ws

            def t(fn, wl=wl):
                it = iter(range(1 << 30))
                return round(timeit(lambda: fn(wl[next(it) % copies]), iters=4 * copies), 1)

            bn = nat.wgemm_tile_n(cfg)
            if N % bn:
                continue
            tiles = N // bn * ((M + 255) // 256)
            if name == "gate_up":
                mt = (M + 255) // 256
                wsb = torch.empty(mt * N * 256, device="cuda", dtype=torch.float32)
                tick = torch.zeros(2 * mt * (N // bn) + 1, device="cuda", dtype=torch.int32)
                for S in (1, 2):
                    row[f"w{cfg}_glu_S{S}"] = t(lambda w: nat.wgemm_glu(x, w, S, cfg, wsb, tick))
                assert int(tick.sum()) == 0
                ref = ops.reference.silu_mul((x.float() @ ws[0].float().T).bfloat16(), interleaved=True)
                got = nat.wgemm_glu(x, wl[0], 2, cfg, wsb, tick)
                row[f"w{cfg}_glu_err"] = round(float((got.float() - ref).abs().max()), 4)
            elif name == "lm_head":
                row[f"w{cfg}_argmax"] = t(lambda w: nat.wgemm_argmax_val(x, w, N, cfg))
            else:
                for S in (1, 2, 4, 7, 8, 14, 16):
                    if K % (S * 64) or tiles * S > 512 or tiles * S < 96:
                        continue
                    row[f"w{cfg}_S{S}"] = t(lambda w: nat.wgemm(x, w, S, cfg))
        print(json.dumps(row), flush=True)
        del wsp
