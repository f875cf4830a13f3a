"""A/B of the batch-256 decode projections on row-major vs stage-tiled weights (round 6).
mgemm.hip streams each weight tile as BN rows x 128 B per 64-deep K stage; on row-major
[N, K] weights those are BN scattered 128-B pieces at a K x 2 B stride, on the tiled copy
([N / BN][K / 64][BN][64]) one contiguous BN x 128 B run.  Same kernel otherwise (bit-exact
outputs); weights cycle through copies past the 256 MB MALL; the two arms alternate
(rounds x iters) so clock / thermal drift hits both.

python scripts/tiled_weight_ab.py [rounds] [iters] [M]
"""
from __future__ import annotations

import json
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from docqa_amd import ops  # noqa: E402


def tile_w(w: torch.Tensor, bn: int) -> torch.Tensor:
    N, K = w.shape
    return w.view(N // bn, bn, K // 64, 64).permute(0, 2, 1, 3).contiguous().view(N, K)


def timeit(fn, iters: int) -> float:
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main() -> None:
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    M = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    assert ops.load_native()
    nat = torch.ops.docqa
    g = torch.Generator(device="cuda").manual_seed(0)
    # (name, N, K, S, cfg row-major, cfg tiled, BN, kind)
    projs = [("qkv", 6144, 4096, 4, 2, 11, 128, "slab"), ("o", 4096, 4096, 4, 7, 13, 64, "slab"),
             ("gate_up", 28672, 4096, 1, 2, 11, 128, "glu"), ("down", 4096, 14336, 8, 2, 11, 128, "slab"),
             ("lm_head", 128256, 4096, 1, 6, 14, 256, "argmax")]
    for name, N, K, S, c0, c1, bn, kind in projs:
        x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
        ncopy = max(2, (768 << 20) // (N * K * 2) + 1)
        ws = [(torch.randn(N, K, device="cuda", generator=g) * 0.02).to(torch.bfloat16) for _ in range(ncopy)]
        wt = [tile_w(w, bn) for w in ws]

        def run(c, wl):
            if kind == "glu":
                return lambda i: nat.mgemm_glu(x, wl[i % ncopy], c)
            if kind == "argmax":
                return lambda i: nat.mgemm_argmax(x, wl[i % ncopy], N, c)
            return lambda i: nat.mgemm(x, wl[i % ncopy], S, c)
        a, b = run(c0, ws), run(c1, wt)
        exact = bool(torch.equal(a(0), b(0)))
        for f in (a, b):
            for i in range(3):
                f(i)
        torch.cuda.synchronize()
        ta, tb = [], []
        for _ in range(rounds):
            ta.append(timeit(a, iters))
            tb.append(timeit(b, iters))
        ma, mb = statistics.median(ta), statistics.median(tb)
        print(json.dumps({"proj": name, "M": M, "N": N, "K": K, "S": S, "cfg_rowmajor": c0, "cfg_tiled": c1,
                          "exact": exact, "rowmajor_us": round(ma, 1), "tiled_us": round(mb, 1),
                          "tiled_over_rowmajor": round(mb / ma, 3), "rowmajor_all": [round(t, 1) for t in ta],
                          "tiled_all": [round(t, 1) for t in tb]}), flush=True)
        del ws, wt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
