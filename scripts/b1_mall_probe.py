"""Batch-1 decode projections from HBM vs from the MALL: how much would a weight prefetch,
issued while the (bandwidth-idle) batch-1 attention runs, buy the next projection?

Per projection: time the skinny decode GEMM (dgemm.hip at ops.decode_plan's split) on M = 1
(a) cold -- weights rotated over > 1 GB of copies -- and (b) right after a read-only touch
of the same weights (a sum over them), timing the GEMM alone with events.

Usage: python scripts/b1_mall_probe.py
"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

from docqa_amd import ops

ops.load_native()


def main():
    for name, N, K in [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)]:
        nb = N * K * 2
        copies = max(2, (1 << 30) // nb + 1)
        ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(copies)]
        x = torch.randn(1, K, device="cuda", dtype=torch.bfloat16)
        S, t = ops.decode_plan(1, N, K)
        if not S:
            continue
        f = lambda w: ops.dgemm_partial(x, w, S, t)
        for w in ws[:2]:
            f(w)
        torch.cuda.synchronize()
        res = {"proj": name, "MB": round(nb / 1e6, 1), "S": S, "tile_rows": t}
        for mode in ("cold", "touched"):
            ts = []
            for i in range(4 * copies):
                w = ws[i % copies]
                if mode == "touched":
                    w.view(torch.int16).sum(dtype=torch.int64)   # read every byte once
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                f(w)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            ts.sort()
            res[f"{mode}_us_p50"] = round(ts[len(ts) // 2], 2)
            res[f"{mode}_TBps"] = round(nb / ts[len(ts) // 2] / 1e6, 2)
        print(json.dumps(res), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
