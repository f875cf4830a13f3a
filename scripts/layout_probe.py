"""Decode-GEMM layout probe (round 6): does a padded row stride of X / W change the
batch-256 projections' time?  Every stage of mgemm.hip reads 256 rows (X) and 128 rows (W)
of 128 B at a row stride of K x 2 B = 8 or 28 KB -- a power of two times 4 KB -- so, if the
L2 / HBM channel hash is a plain function of the low address bits, all of a stage's lines
land on ONE channel.  Pads of 64-128 elements spread them.

Weights are cycled through enough copies that every call streams them from HBM (as the
decode step does: 15 GB per step), X is hot (written by the previous kernel).

python scripts/layout_probe.py [iters]
"""
from __future__ import annotations

import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from docqa_amd import ops  # noqa: E402


def timeit(fn, iters: int) -> float:
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main() -> None:
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    assert ops.load_native()
    nat = torch.ops.docqa
    M = 256
    shapes = [("qkv", 6144, 4096, 4, 2, False), ("o", 4096, 4096, 4, 7, False),
              ("down", 4096, 14336, 8, 2, False), ("gate_up", 28672, 4096, 1, 2, True)]
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, N, K, S, cfg, glu in shapes:
        res = {"proj": name, "M": M, "N": N, "K": K, "S": S, "cfg": cfg}
        ncopy = max(2, (768 << 20) // (N * K * 2) + 1)
        for xpad in (0, 64):
            xb = torch.randn(M, K + xpad, device="cuda", generator=g).to(torch.bfloat16)
            x = xb[:, :K]
            for wpad in (0, 64):
                ws = [(torch.randn(N, K + wpad, device="cuda", generator=g) * 0.02).to(torch.bfloat16)[:, :K]
                      for _ in range(ncopy)]
                if xpad == 0 and wpad == 0:
                    if glu:
                        ref = nat.mgemm_glu(x.contiguous(), ws[0].contiguous(), cfg)
                        base = timeit(lambda i: nat.mgemm_glu(x, ws[i % ncopy], cfg), iters)
                    else:
                        ref = nat.mgemm(x.contiguous(), ws[0].contiguous(), S, cfg)
                        base = timeit(lambda i: nat.mgemm(x, ws[i % ncopy], S, cfg), iters)
                    res["base_us"] = round(base, 1)
                out = nat.mgemm_ld(x, ws[0], S, cfg, glu)
                res[f"exact_x{xpad}_w{wpad}"] = bool(torch.equal(out, ref))
                t = timeit(lambda i: nat.mgemm_ld(x, ws[i % ncopy], S, cfg, glu), iters)
                res[f"x{xpad}_w{wpad}_us"] = round(t, 1)
                del ws
                torch.cuda.empty_cache()
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
