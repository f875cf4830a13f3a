"""Decode-sized GEMMs (M = batch bucket): the 256 x 256 8-phase kernel with split-K fp32
slabs (pgemm.hip EPI_PARTIAL) vs the mid-M kernel (mgemm.hip, ops.mid_plan) on the Llama-3-8B
projections, weights rotated through > 1 GB of copies so every call streams them from HBM
(as a decode step does), interleaved rounds in one process.

Usage: python scripts/pgemm_decode_probe.py [M ...]
"""
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from docqa_amd import ops  # noqa: E402

PROJ = {"qkv": (6144, 4096), "o": (4096, 4096), "down": (4096, 14336), "gate_up": (28672, 4096)}


def main():
    assert ops.load_native()
    Ms = [int(a) for a in sys.argv[1:]] or [256, 384, 512]
    for M in Ms:
        for name, (N, K) in PROJ.items():
            x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
            nrot = max(2, (1 << 30) // (N * K * 2))
            ws = [((torch.rand(N, K, device="cuda") * 2 - 1) / K ** 0.5).to(torch.bfloat16) for _ in range(nrot)]
            Sm, cm = ops.mid_plan(M, N, K)
            cands = {}
            if Sm:
                cands[f"mgemm_S{Sm}_c{cm}"] = lambda w, Sm=Sm, cm=cm: ops.mgemm_partial(x, w, Sm, cm)
            tiles = ((M + 255) // 256) * (N // 256)
            for S in (1, 2, 4, 8, 16):
                if K % (S * 128) == 0 and tiles * S <= 512 and tiles * S >= 64:
                    cands[f"pgemm_S{S}"] = lambda w, S=S: torch.ops.docqa.pgemm_partial(x, w, S)
            t = {k: [] for k in cands}
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            for _ in range(5):
                for k, f in cands.items():
                    f(ws[0])
                    torch.cuda.synchronize()
                    ev[0].record()
                    for w in ws:
                        f(w)
                    ev[1].record()
                    torch.cuda.synchronize()
                    t[k].append(ev[0].elapsed_time(ev[1]) * 1e3 / len(ws))
            out = {"M": M, "proj": name, "N": N, "K": K}
            for k, v in t.items():
                us = statistics.median(v)
                out[k] = {"us": round(us, 1), "TBps": round(N * K * 2 / us / 1e6, 2)}
            print(json.dumps(out), flush=True)
            del ws


if __name__ == "__main__":
    main()
