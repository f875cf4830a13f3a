"""Prefill GEMM probe: the hand-written 256 x 256 kernel (pgemm.hip), the 128 x 128 kernel
(gemm.hip) and hipBLASLt (F.linear) on the Llama prefill projection shapes, interleaved
rounds in one process (cdna_hip_programming.md §5.4 rule 24), uniform random operands.

Usage: python scripts/pgemm_probe.py [M ...]   -> one JSON line per (M, projection)
"""
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from docqa_amd import ops  # noqa: E402

PROJ = {  # name: (N, K, epi) for Llama-3-8B (TP=1) and 70B at TP=8
    "qkv": (6144, 4096, 0), "o": (4096, 4096, 0), "gate_up": (28672, 4096, 1), "down": (4096, 14336, 0),
    "70b_qkv": (1280, 8192, 0), "70b_o": (8192, 1024, 0), "70b_gate_up": (7168, 8192, 1), "70b_down": (8192, 3584, 0),
    "lm_head": (128256, 4096, 0),
}
ONLY = [p for p in os.environ.get("PROBE_PROJ", "").split(",") if p]   # default: all but lm_head


def timeit(fn, reps=10):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) * 1e3 / reps


def main():
    assert ops.load_native()
    Ms = [int(a) for a in sys.argv[1:]] or [16384, 4096, 1024]
    for M in Ms:
        for name, (N, K, epi) in PROJ.items():
            if (ONLY and name not in ONLY) or (not ONLY and name == "lm_head"):
                continue
            x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
            w = ((torch.rand(N, K, device="cuda") * 2 - 1) / K ** 0.5).to(torch.bfloat16)
            if epi:
                lib = lambda: ops.silu_mul(F.linear(x, w), interleaved=True)
                mine = lambda: torch.ops.docqa.pgemm(x, w, 1)
                small = lambda: ops.silu_mul(torch.ops.docqa.gemm(x, w, None, None, 0), interleaved=True)
            else:
                lib = lambda: F.linear(x, w)
                mine = lambda: torch.ops.docqa.pgemm(x, w, 0)
                small = lambda: torch.ops.docqa.gemm(x, w, None, None, 0)
            r = x.float() @ w.float().t()
            if epi:
                r = ops.reference.silu_mul(r, interleaved=True).float()
            err = (mine().float() - r).abs().max().item() / max(1e-6, r.abs().max().item())
            t = {"pgemm": [], "gemm128": [], "hipblaslt": []}
            for _ in range(5):
                t["pgemm"].append(timeit(mine))
                t["gemm128"].append(timeit(small))
                t["hipblaslt"].append(timeit(lib))
            flops = 2.0 * M * N * K
            out = {"M": M, "proj": name, "N": N, "K": K, "rel_err": round(err, 5)}
            for k, v in t.items():
                med = statistics.median(v)
                out[k + "_us"] = round(med, 1)
                out[k + "_TF"] = round(flops / med / 1e6, 1)
            out["pgemm_vs_lib"] = round(out["hipblaslt_us"] / out["pgemm_us"], 3)
            print(json.dumps(out), flush=True)
            del x, w, r


if __name__ == "__main__":
    main()
