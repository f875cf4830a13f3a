"""Batch-1 decode projections: the register-streaming GEMV (dgemm.hip gemv_kernel) against
the LDS-ring skinny GEMM at its shipped plan (ops.decode_plan), weights rotated past the
256 MB MALL as in a decode step, per Llama-3-8B projection; max |err| vs the fp32 product.

python scripts/gemv_probe.py   -> one JSON line per (projection, variant)"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from docqa_amd import ops  # noqa: E402

SHAPES = [("qkv", 6144, 4096, False), ("o", 4096, 4096, False), ("gate_up", 28672, 4096, True),
          ("down", 4096, 14336, False)]


def timeit(fn, copies, iters=60):
    for i in range(copies):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(iters):
        fn(i % copies)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    assert ops.load_native()
    nat = torch.ops.docqa
    for name, N, K, glu in SHAPES:
        copies = max(2, (768 << 20) // (N * K * 2) + 1)
        ws = [((torch.rand(N, K, device="cuda") * 2 - 1) / K ** 0.5).to(torch.bfloat16) for _ in range(copies)]
        x = (torch.rand(1, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        ref = x.float() @ ws[0].float().t()
        if glu:
            ref = ops.reference.silu_mul(ref.bfloat16(), interleaved=True).float()
        S, t = ops.decode_plan(1, N, K)
        cands = {}
        if glu:
            cands["ring_glu"] = lambda i: nat.dgemm_glu(x, ws[i])
            for R, S2 in ((16, 1),):
                cands[f"gemv_R{R}"] = (lambda i, R=R: nat.gemv(x, ws[i], 1, R, True))
        else:
            cands[f"ring_S{S}_t{t}"] = lambda i: nat.dgemm_partial(x, ws[i], S, t)
            for R in (4, 8, 16):
                for S2 in (1, 2, 4, 7):
                    if K % S2 or (K // S2) % 2048:
                        continue
                    C = K // S2 // 2048
                    if (R, C) not in ((16, 1), (16, 2), (8, 2), (8, 4), (4, 4), (4, 7), (8, 1), (4, 2), (4, 1)):
                        continue
                    cands[f"gemv_R{R}_S{S2}"] = (lambda i, R=R, S2=S2: nat.gemv(x, ws[i], S2, R, False))
        for k, fn in cands.items():
            out = fn(0)
            y = out.float().sum(0) if out.dim() == 3 else out.float()
            err = (y.reshape(ref.shape) - ref).abs().max().item()
            us = timeit(fn, copies)
            print(json.dumps({"proj": name, "variant": k, "us": round(us, 2), "TBps": round(N * K * 2 / us / 1e6, 2),
                              "err": round(err, 5)}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def xn_main():
    """XN mode (input row built in-kernel from 2 fp32 slabs + residual + gamma): every
    workgroup runs the prologue, so fewer, wider workgroups may win."""
    assert ops.load_native()
    nat = torch.ops.docqa
    H = 4096
    Pin = torch.randn(2, 1, H, device="cuda")
    res = torch.randn(1, H, device="cuda").to(torch.bfloat16)
    res2 = torch.empty_like(res)
    gamma = torch.ones(H, device="cuda", dtype=torch.bfloat16)
    for name, N, glu in (("qkv", 6144, False), ("gate_up", 28672, True)):
        copies = max(2, (768 << 20) // (N * H * 2) + 1)
        ws = [((torch.rand(N, H, device="cuda") * 2 - 1) / H ** 0.5).to(torch.bfloat16) for _ in range(copies)]
        cands = {}
        if glu:
            cands["ring_glu_xn"] = lambda i: nat.dgemm_glu_xn(Pin, res, res2, gamma, 1e-5, ws[i])
            cands["gemv_glu_xn_R16"] = lambda i: nat.gemv_xn(Pin, res, res2, gamma, 1e-5, ws[i], 1, 16, True)
        else:
            cands["ring_xn_S2"] = lambda i: nat.dgemm_partial_xn(Pin, res, res2, gamma, 1e-5, ws[i], 2)
            for R, S in ((4, 2), (8, 2), (16, 2), (8, 1), (16, 1)):
                cands[f"gemv_xn_R{R}_S{S}"] = (lambda i, R=R, S=S: nat.gemv_xn(Pin, res, res2, gamma, 1e-5, ws[i], S, R,
                                                                             False))
        for k, fn in cands.items():
            us = timeit(fn, copies)
            print(json.dumps({"proj": name, "variant": k, "us": round(us, 2), "TBps": round(N * H * 2 / us / 1e6, 2)}),
                  flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "xn":
    xn_main()
