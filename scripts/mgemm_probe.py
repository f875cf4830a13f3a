"""Mid-M decode GEMMs (M = 193..512 rows, the bench's batch 256 decode step): hipBLASLt
(F.linear, default heuristics) vs the hand-written 128x128 MFMA GEMM (gemm.hip) vs the
mid-M split-K kernel (mgemm.hip) when built, weights rotating past the 256 MB MALL.
Usage: python scripts/mgemm_probe.py [M ...]"""
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
import os
Ms = [int(a) for a in sys.argv[1:]] or [256]
HOT = os.environ.get("PROBE_HOT", "0") == "1"   # weights NOT rotated past the MALL
res = []
for (name, N, K) in [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096),
                     ("down", 4096, 14336), ("lm_head", 128256, 4096)]:
    nb = N * K * 2
    copies = 1 if HOT else max(2, (1 << 30) // nb + 1)
    ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(copies)]
    for M in Ms:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        row = {"proj": name, "M": M, "weights_MB": round(nb / 2 ** 20, 1)}
        it = iter(range(1 << 30))
        row["hipblaslt_us"] = round(timeit(lambda: F.linear(x, ws[next(it) % copies]), iters=4 * copies), 1)
        it = iter(range(1 << 30))
        row["gemm128_us"] = round(timeit(lambda: nat.gemm(x, ws[next(it) % copies], None, None, 0),
                                         iters=4 * copies), 1)
        ref = F.linear(x.float(), ws[0].float())
        got = nat.gemm(x, ws[0], None, None, 0).float()
        row["gemm128_err"] = float((got - ref).abs().max() / ref.abs().max())
        if hasattr(nat, "mgemm"):
            for bn in [int(c) for c in os.environ.get("PROBE_CFGS", "2,5,6").split(",")]:
                for S in (1, 2, 4, 7, 8, 14, 16):
                    BNc = 256 if 3 <= bn <= 6 else 64 if bn == 7 else 128
                    if K % (S * 128) or N % BNc or (S > 1 and name in ("gate_up", "lm_head")):
                        continue
                    if S > 1 and (N // BNc) * S > 512:
                        continue
                    it = iter(range(1 << 30))
                    try:
                        row[f"c{bn}_S{S}"] = round(timeit(lambda: nat.mgemm(x, ws[next(it) % copies], S, bn),
                                                           iters=4 * copies), 1)
                    except RuntimeError as e:
                        row[f"c{bn}_S{S}"] = str(e)[:60]
                try:
                    if name == "gate_up":
                        it = iter(range(1 << 30))
                        row[f"glu{bn}"] = round(timeit(lambda: nat.mgemm_glu(x, ws[next(it) % copies], bn),
                                                       iters=4 * copies), 1)
                    if name == "lm_head":
                        it = iter(range(1 << 30))
                        row[f"argmax{bn}"] = round(timeit(lambda: nat.mgemm_argmax(x, ws[next(it) % copies], N, bn),
                                                          iters=4 * copies), 1)
                except RuntimeError as e:
                    row[f"fused{bn}"] = str(e)[:60]
        row["hbm_TBs_at_hipblaslt"] = round(nb / row["hipblaslt_us"] / 1e6, 2)
        print(json.dumps(row), flush=True)
        res.append(row)
    del ws
    torch.cuda.empty_cache()
