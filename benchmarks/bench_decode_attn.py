"""Paged decode attention bandwidth on realistic (HBM-resident) caches: K/V caches rotate
over >= 1 GiB of copies so repeated calls are not served from the 256 MB MALL, as in a real
decode step where every layer's cache is read once.  Knobs are read from the environment
(DOCQA_DECODE_WG_TARGET, DOCQA_DECODE_U); run one process per setting."""
from __future__ import annotations

import json
import math
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

from benchmarks.bench_kernels import timeit


MIX = os.environ.get("MIX", "uniform")      # uniform | random | sorted | lpt context lengths


def main():
    from docqa_amd import ops

    assert ops.load_native()
    nat = torch.ops.docqa
    res = []
    Hq, Hkv, D, BS = int(os.environ.get("HQ", "32")), 8, 128, 64   # HQ=64: Llama-3-70B (G=8)
    shapes = [(64, 640), (64, 1024), (32, 640), (8, 1024), (1, 4096)]
    if os.environ.get("SHAPES"):
        shapes = [tuple(int(v) for v in x.split("x")) for x in os.environ["SHAPES"].split(",")]
    for (B, ctx) in shapes:
        maxb = (ctx * (2 if MIX != "uniform" else 1) + BS - 1) // BS
        nbytes = 2 * B * maxb * Hkv * BS * D * 2
        copies = max(2, (1 << 30) // nbytes + 1)
        caches = [(torch.randn(B * maxb, Hkv, BS, D, device="cuda", dtype=torch.bfloat16),
                   torch.randn(B * maxb, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)) for _ in range(copies)]
        bt = torch.arange(B * maxb, device="cuda", dtype=torch.int32).view(B, maxb)
        cl = torch.full((B,), ctx, device="cuda", dtype=torch.int32)
        if MIX != "uniform":
            # same mean context, lengths spread over [0.4, 1.6] x ctx (a RAG batch), in
            # random order or longest first (LPT dispatch order)
            g = torch.Generator().manual_seed(0)
            lens = (ctx * (0.4 + 1.2 * torch.rand(B, generator=g))).int().clamp(1, maxb * BS)
            if MIX == "sorted":   # the rows themselves sorted (no order input)
                lens = lens.sort(descending=True).values
            cl = lens.to(torch.int32).cuda()
        q = torch.randn(B, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
        # MIX=lpt: random lengths, dispatched longest first through the kernel's order input
        order = torch.argsort(cl.cpu(), descending=True).int().cuda() if MIX == "lpt" else None
        it = iter(range(1 << 30))

        def run():
            kc, vc = caches[next(it) % copies]
            return nat.paged_decode(q, kc, vc, bt, cl, Hq, 2048 if ctx < 2048 else 4096, 1 / math.sqrt(D), order)
        t = timeit(run, iters=4 * copies)
        kv = 2 * int(cl.sum()) * Hkv * D * 2
        res.append({"B": B, "ctx": ctx, "mix": MIX, "us": round(t, 1), "kv_TBps": round(kv / t / 1e6, 2)})
        del caches
        torch.cuda.empty_cache()
    print(json.dumps({"mfma": os.environ.get("DOCQA_DECODE_MFMA", "1"), "nsr": os.environ.get("DOCQA_DECODE_NSR", "4"),
                      "wg_target": os.environ.get("DOCQA_DECODE_WG_TARGET", "512"),
                      "U": os.environ.get("DOCQA_DECODE_U", "2"), "rows": res}), flush=True)


if __name__ == "__main__":
    main()
