"""Mid-M prefill GEMM probe (pgemm below hipBLASLt at M = 1k-4k and at the
70B TP-8 shapes): every hand-written candidate vs hipBLASLt per (M, projection), medians
of interleaved rounds:
  pgemm   -- 256 x 256 tiles (pgemm.hip)
  gemm128 -- 128 x 128 tiles (gemm.hip)
  mgemm_c -- 256-row m-tiles x (128 | 256 | 64)-row weight tiles, K unsplit (mgemm.hip cfg c)
  pgS     -- pgemm split-K slabs (pgemm_partial, S = 2) + the fp32 slab sum (what a fused
             split-K consumer would pay)
  routed  -- what the prefill forward runs for the projection (ops.prefill_route, the plan
             logic of models/llama.py: split-K plans timed as their slabs alone, since the
             RoPE / add+RMSNorm consumer that sums them runs either way); "route" names it
             (scripts/prefill_mid_probe.py times the same WITH the consumers)
Usage: python scripts/pgemm_mid_probe.py [M ...]   -> one JSON line per (M, projection)"""
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from docqa_amd import ops  # noqa: E402

PROJ = {
    "qkv": (6144, 4096, 0), "o": (4096, 4096, 0), "gate_up": (28672, 4096, 1), "down": (4096, 14336, 0),
    "70b_qkv": (1280, 8192, 0), "70b_o": (8192, 1024, 0), "70b_gate_up": (7168, 8192, 1), "70b_down": (8192, 3584, 0),
}


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
    nat = torch.ops.docqa
    Ms = [int(a) for a in sys.argv[1:]] or [512, 1024, 2048, 4096]
    for M in Ms:
        only = os.environ.get("PROBE_PROJ", "")
        for name, (N, K, epi) in PROJ.items():
            if only and name not in only.split(","):
                continue
            x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
            w = ((torch.rand(N, K, device="cuda") * 2 - 1) / K ** 0.5).to(torch.bfloat16)
            c = {}
            route, rfn = ops.prefill_route(M, N, K, glu=bool(epi), down=name.endswith("down"))
            c["routed"] = lambda: rfn(x, w)
            if epi:
                c["hipblaslt"] = lambda: ops.silu_mul(F.linear(x, w), interleaved=True)
                if N % 256 == 0:
                    c["pgemm"] = lambda: nat.pgemm(x, w, 1)
                c["mgemm_2"] = lambda: nat.mgemm_glu(x, w, 2)
                c["gemm128"] = lambda: nat.gemm(x, w, None, None, 4)
                c["mgemm_6"] = lambda: nat.mgemm_glu(x, w, 6)
            else:
                c["hipblaslt"] = lambda: F.linear(x, w)
                if N % 256 == 0:
                    c["pgemm"] = lambda: nat.pgemm(x, w, 0)
                    for S in (2, 4, 8, 16):
                        if K % (128 * S) == 0 and (S == 2 or N < 4096):
                            c[f"pgS{S}"] = (lambda S=S: nat.pgemm_partial(x, w, S).sum(0))
                            c[f"pgS{S}_only"] = (lambda S=S: nat.pgemm_partial(x, w, S))
                c["gemm128"] = lambda: nat.gemm(x, w, None, None, 0)
                for cfg in (2, 6, 7):
                    if N % nat.mgemm_tile_n(cfg) == 0:
                        c[f"mgemm_{cfg}"] = (lambda cfg=cfg: nat.mgemm(x, w, 1, cfg))
            # mid-M split-K slab plans (the consumer that sums them runs anyway: RoPE / add +
            # RMSNorm, or for gate|up the SwiGLU of the slab sum); "_only" = the slabs alone
            for cfg in (2, 7):
                for S in (2, 3, 4, 8):
                    if N % nat.mgemm_tile_n(cfg) == 0 and K % (S * 128) == 0:
                        c[f"mS{S}c{cfg}_only"] = (lambda S=S, cfg=cfg: nat.mgemm(x, w, S, cfg))
            r = x.float() @ w.float().t()
            if epi:
                r = ops.reference.silu_mul(r, interleaved=True).float()
            errs = {}
            for k, fn in c.items():
                try:
                    y = fn().float()
                    if k.endswith("_only") or (k == "routed" and y.dim() == 3):
                        y = y.sum(0)
                        if epi and y.shape[-1] == N:
                            y = ops.reference.silu_mul(y.to(torch.bfloat16).float(), interleaved=True).float()
                    errs[k] = round((y - r).abs().max().item() / max(1e-6, r.abs().max().item()), 5)
                except Exception as e:  # noqa: BLE001 -- a shape a candidate does not take
                    errs[k] = f"n/a: {str(e).splitlines()[0][:60]}"
            t = {k: [] for k in c if not isinstance(errs[k], str)}
            for _ in range(5):
                for k in t:
                    t[k].append(timeit(c[k]))
            flops = 2.0 * M * N * K
            out = {"M": M, "proj": name, "N": N, "K": K}
            for k, v in t.items():
                med = statistics.median(v)
                out[k + "_us"] = round(med, 1)
                out[k + "_TF"] = round(flops / med / 1e6, 1)
            hand = [k for k in t if k not in ("hipblaslt", "routed") and not k.endswith("_only")]
            best = min(hand, key=lambda k: out[k + "_us"])
            out["best"] = best
            out["best_vs_lib"] = round(out["hipblaslt_us"] / out[best + "_us"], 3)
            # slab plans priced with their consumer's extra slab reads (S fp32 slabs at ~5 TB/s,
            # minus the one bf16 pass a plain consumer reads anyway)
            slab = {k: out[k + "_us"] + (int(k[2:k.index("c")]) * 4 - 2) * M * N / 5e6
                    for k in t if k.startswith("mS")}
            if slab:
                bs = min(slab, key=slab.get)
                out["best_slab"], out["best_slab_priced_us"] = bs, round(slab[bs], 1)
                out["best_slab_vs_lib"] = round(out["hipblaslt_us"] / slab[bs], 3)
            out["route"] = route
            if "routed" in t:
                out["routed_vs_lib"] = round(out["hipblaslt_us"] / out["routed_us"], 3)
            out["errs"] = errs
            print(json.dumps(out), flush=True)
            del x, w, r


if __name__ == "__main__":
    main()
