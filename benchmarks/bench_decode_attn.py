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


def main():
    from docqa_amd import ops

    assert ops.load_native()
    nat = torch.ops.docqa
    res = []
    Hq, Hkv, D, BS = 32, 8, 128, 64
    shapes = [(64, 640), (64, 1024), (32, 640), (8, 1024), (1, 4096)]
    if os.environ.get("SHAPES"):
        shapes = [tuple(int(v) for v in x.split("x")) for x in os.environ["SHAPES"].split(",")]
    for (B, ctx) in shapes:
        maxb = (ctx + BS - 1) // BS
        nbytes = 2 * B * maxb * Hkv * BS * D * 2
        copies = max(2, (1 << 30) // nbytes + 1)
        caches = [(torch.randn(B * maxb, Hkv, BS, D, device="cuda", dtype=torch.bfloat16),
                   torch.randn(B * maxb, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)) for _ in range(copies)]
        bt = torch.arange(B * maxb, device="cuda", dtype=torch.int32).view(B, maxb)
        cl = torch.full((B,), ctx, device="cuda", dtype=torch.int32)
        q = torch.randn(B, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
        it = iter(range(1 << 30))

        def run():
            kc, vc = caches[next(it) % copies]
            return nat.paged_decode(q, kc, vc, bt, cl, Hq, 2048 if ctx < 2048 else 4096, 1 / math.sqrt(D))
        t = timeit(run, iters=4 * copies)
        res.append({"B": B, "ctx": ctx, "us": round(t, 1), "kv_TBps": round(2 * B * ctx * Hkv * D * 2 / t / 1e6, 2)})
        del caches
        torch.cuda.empty_cache()
    print(json.dumps({"mfma": os.environ.get("DOCQA_DECODE_MFMA", "1"), "nsr": os.environ.get("DOCQA_DECODE_NSR", "4"),
                      "wg_target": os.environ.get("DOCQA_DECODE_WG_TARGET", "512"),
                      "U": os.environ.get("DOCQA_DECODE_U", "2"), "rows": res}), flush=True)


if __name__ == "__main__":
    main()
