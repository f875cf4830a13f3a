"""Transfer floor of the batch-256 decode GEMM's ring (round 6): the
same mgemm.hip schedule (a) as shipped, (b) without its MFMAs, (c) without MFMAs and
fragment reads -- only the LDS-DMA ring, its counted waits and barriers -- and (d) a
32-deep x 6-slot ring (5 stages, 120 KB in flight) without compute.  If (c) is close to
(a), the projection is bound by moving its bytes (W from HBM once + X re-read from L2 by
every weight tile), not by the MFMA / LDS-read side; (d) says whether more bytes in flight
would move that floor.  Weights cycle through copies past the 256 MB MALL (cold, as in the
decode step).

python scripts/mgemm_floor_probe.py [iters]
"""
from __future__ import annotations

import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from docqa_amd import ops  # noqa: E402


def timeit(fn, iters: int) -> float:
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main() -> None:
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    only = set(sys.argv[2].split(",")) if len(sys.argv) > 2 else set()
    assert ops.load_native()
    nat = torch.ops.docqa
    M = 256
    g = torch.Generator(device="cuda").manual_seed(0)
    shapes = [("gate_up", 28672, 4096, 1, True), ("qkv", 6144, 4096, 4, False), ("down", 4096, 14336, 8, False),
              ("down_S4", 4096, 14336, 4, False), ("qkv_S1", 6144, 4096, 1, False)]
    for name, N, K, S, glu in shapes:
        x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
        ncopy = max(2, (768 << 20) // (N * K * 2) + 1)
        ws = [(torch.randn(N, K, device="cuda", generator=g) * 0.02).to(torch.bfloat16) for _ in range(ncopy)]
        wmb = N * K * 2 / 1e6
        tiles = N // 128 * S
        xmb_per_wg = M * (K // S) * 2 / 1e6
        res = {"proj": name, "N": N, "K": K, "S": S, "weights_MB": round(wmb, 1), "workgroups": tiles,
               "bytes_per_wg_MB": round(xmb_per_wg + wmb / tiles, 3)}
        # stage-tiled weight copies: [N / 128][K / 64][128][64] (one 16 KiB run per stage)
        wts = [w.view(N // 128, 128, K // 64, 64).permute(0, 2, 1, 3).contiguous().view(N, K) for w in ws]
        for cfg, label, wl in ((2, "shipped", ws), (8, "no_mfma", ws), (9, "dma_only", ws),
                               (10, "dma_only_6x32", ws), (11, "tiledW", wts), (12, "tiledW_dma_only", wts)):
            if only and label not in only:
                continue
            if glu:
                fn = lambda i, c=cfg, wl=wl: nat.mgemm_glu(x, wl[i % ncopy], c)
            else:
                fn = lambda i, c=cfg, wl=wl: nat.mgemm(x, wl[i % ncopy], S, c)
            t = timeit(fn, iters)
            res[label + "_us"] = round(t, 1)
            res[label + "_GBps_per_wg"] = round(res["bytes_per_wg_MB"] * 1e3 / t, 1)
        a = nat.mgemm_glu(x, ws[0], 2) if glu else nat.mgemm(x, ws[0], S, 2)
        b = nat.mgemm_glu(x, wts[0], 11) if glu else nat.mgemm(x, wts[0], S, 11)
        res["tiledW_exact"] = bool(torch.equal(a, b))
        del wts
        print(json.dumps(res), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
