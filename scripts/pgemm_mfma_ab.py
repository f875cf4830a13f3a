"""Prefill GEMM MFMA-shape A/B (prefill efficiency under the power cap):
the 256 x 256 kernel with 16x16x32 vs 32x32x16 MFMAs (pgemm.hip Tile<MF32>; same tiles, LDS
layout and schedule -- the 32x32x16 form reads half the operand registers per FLOP), each
run back to back for ~SECONDS so the clock settles at the power cap, on the headline
prefill's Llama-3-8B shapes.  Run it under scripts/power_probe.py for the clock.

python scripts/pgemm_mfma_ab.py [M] [seconds]   -> one JSON line per (shape, variant)"""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from docqa_amd import ops  # noqa: E402

SHAPES = [("qkv", 6144, 4096, 0), ("o", 4096, 4096, 0), ("gate_up", 28672, 4096, 1), ("down", 4096, 14336, 0)]


def main():
    assert ops.load_native()
    nat = torch.ops.docqa
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
    for name, N, K, epi in SHAPES:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        for rnd in range(2):
            for mf in (0, 1):
                nat.pgemm_mf(x, w, epi, mf)
                torch.cuda.synchronize()
                n, t0 = 0, time.time()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                while time.time() - t0 < secs:
                    for _ in range(20):
                        nat.pgemm_mf(x, w, epi, mf)
                    n += 20
                    torch.cuda.synchronize()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / n
                print(json.dumps({"proj": name, "M": M, "N": N, "K": K, "mfma": "32x32x16" if mf else "16x16x32",
                                  "round": rnd, "us": round(us, 1), "TFLOPs": round(2 * M * N * K / us / 1e6, 1)}),
                      flush=True)


if __name__ == "__main__":
    main()
