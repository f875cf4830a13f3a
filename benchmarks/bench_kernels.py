"""Kernel micro-benchmarks on one MI355X: each hand-written HIP kernel against the best
library/PyTorch path for the same op, interleaved in one process (guide §5.4 rule 24),
random data.  One JSON line per kernel group."""
from __future__ import annotations

import json
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch
import torch.nn.functional as F


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def bench_dgemm(nat):
    """Decode projections of Llama-3-8B (M = decode batch): ours vs hipBLASLt (F.linear).
    Weights rotate through >= 1 GiB of copies so neither path is served from the 256 MB
    MALL, as in a real decode step where every layer's weights are read once."""
    rows = []
    for (name, N, K) in [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096),
                         ("down", 4096, 14336), ("lm_head", 128256, 4096)]:
        nb = N * K * 2
        copies = max(2, (1 << 30) // nb + 1)
        ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(copies)]
        for M in (1, 16, 32, 64):
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            it = iter(range(1 << 30))
            t_ours = timeit(lambda: nat.dgemm(x, ws[next(it) % copies], 0), iters=4 * copies)
            t_lib = timeit(lambda: F.linear(x, ws[next(it) % copies]), iters=4 * copies)
            rows.append({"proj": name, "M": M, "N": N, "K": K, "ours_us": round(t_ours, 1),
                         "hipblaslt_us": round(t_lib, 1), "ours_TBps": round(nb / t_ours / 1e6, 2),
                         "hipblaslt_TBps": round(nb / t_lib / 1e6, 2)})
        if name == "gate_up":   # fused SwiGLU decode GEMM vs hipBLASLt + silu_mul kernel
            for M in (1, 16, 32, 64):
                x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
                it = iter(range(1 << 30))
                t_ours = timeit(lambda: nat.dgemm_glu(x, ws[next(it) % copies]), iters=4 * copies)
                t_lib = timeit(lambda: nat.silu_mul(F.linear(x, ws[next(it) % copies]), True), iters=4 * copies)
                rows.append({"proj": "gate_up+swiglu", "M": M, "N": N, "K": K, "ours_us": round(t_ours, 1),
                             "hipblaslt_plus_silu_us": round(t_lib, 1), "ours_TBps": round(nb / t_ours / 1e6, 2)})
        if "--sweep" in sys.argv and N <= 8192:
            x = torch.randn(64, K, device="cuda", dtype=torch.bfloat16)
            for S in (1, 2, 4, 8, 16):
                if K % S or (K // S) % 512:
                    continue
                it = iter(range(1 << 30))
                t = timeit(lambda: nat.dgemm(x, ws[next(it) % copies], S), iters=4 * copies)
                rows.append({"proj": name, "M": 64, "S": S, "ours_us": round(t, 1)})
        del ws
        torch.cuda.empty_cache()
    return rows


def main():
    from docqa_amd import ops

    assert ops.load_native()
    nat = torch.ops.docqa
    out = {}
    if "--only-dgemm" in sys.argv:
        print(json.dumps({"dgemm": bench_dgemm(nat)}), flush=True)
        return
    out["dgemm"] = bench_dgemm(nat)
    # ---- fused GEMM (encoder shapes): ours vs hipBLASLt linear + separate bias/GELU kernel
    rows = []
    for (M, N, K, epi) in [(16384, 1536, 384, 2), (16384, 384, 1536, 3), (16384, 1152, 384, 1),
                           (8192, 3072, 768, 2), (8192, 768, 3072, 3), (8192, 4096, 4096, 0)]:
        a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
        b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
        r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        bias = b if epi else None
        res = r if epi == 3 else None
        t_ours = timeit(lambda: nat.gemm(a, w, bias, res, epi))

        def lib():
            y = F.linear(a, w)
            if epi:
                y = nat.bias_act(y, b, res, epi == 2)
            return y
        t_lib = timeit(lib)
        fl = 2 * M * N * K
        rows.append({"M": M, "N": N, "K": K, "epi": epi, "ours_us": round(t_ours, 1),
                     "hipblaslt_plus_epilogue_us": round(t_lib, 1),
                     "ours_tflops": round(fl / t_ours / 1e6, 1)})
    out["gemm_fused"] = rows
    # ---- prefill attention: ours vs torch SDPA (flash/aotriton) on the same packed batch
    rows = []
    for (B, L, Hq, Hkv, D) in [(64, 512, 32, 8, 128), (8, 2048, 32, 8, 128), (256, 128, 12, 12, 32)]:
        T = B * L
        qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
        cu = torch.arange(0, T + 1, L, device="cuda", dtype=torch.int32)
        causal = D == 128
        t_ours = timeit(lambda: nat.flash_prefill(qkv, cu, L, Hq, Hkv, D, 1 / math.sqrt(D), causal))
        x = qkv.view(B, L, Hq + 2 * Hkv, D)
        q = x[:, :, :Hq].transpose(1, 2)
        k = x[:, :, Hq:Hq + Hkv].transpose(1, 2).repeat_interleave(Hq // Hkv, 1)
        v = x[:, :, Hq + Hkv:].transpose(1, 2).repeat_interleave(Hq // Hkv, 1)
        t_sdpa = timeit(lambda: F.scaled_dot_product_attention(q, k, v, is_causal=causal))
        fl = 4 * B * Hq * L * L * D / (2 if causal else 1)
        rows.append({"B": B, "L": L, "Hq": Hq, "D": D, "causal": causal, "ours_us": round(t_ours, 1),
                     "torch_sdpa_us": round(t_sdpa, 1), "ours_tflops": round(fl / t_ours / 1e6, 1)})
    out["flash_prefill"] = rows
    # ---- decode attention: bandwidth of KV streaming
    rows = []
    for (B, ctx) in [(64, 640), (1, 4096), (256, 1024)]:
        Hq, Hkv, D, BS = 32, 8, 128, 64
        maxb = (ctx + BS - 1) // BS
        kc = torch.randn(B * maxb, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        bt = torch.arange(B * maxb, device="cuda", dtype=torch.int32).view(B, maxb)
        cl = torch.full((B,), ctx, device="cuda", dtype=torch.int32)
        q = torch.randn(B, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: nat.paged_decode(q, kc, vc, bt, cl, Hq, maxb * BS, 1 / math.sqrt(D)))
        bytes_ = 2 * B * ctx * Hkv * D * 2
        rows.append({"B": B, "ctx": ctx, "us": round(t, 1), "kv_TBps": round(bytes_ / t / 1e6, 2)})
    out["paged_decode"] = rows
    # ---- norms / elementwise (decode-sized and prefill-sized)
    rows = []
    for T in (64, 32768):
        x = torch.randn(T, 4096, device="cuda", dtype=torch.bfloat16)
        r = torch.randn_like(x)
        w = torch.ones(4096, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: nat.add_rmsnorm(x, r, w, 1e-5))
        gu = torch.randn(T, 28672, device="cuda", dtype=torch.bfloat16)
        t2 = timeit(lambda: nat.silu_mul(gu))
        rows.append({"T": T, "add_rmsnorm_us": round(t, 1), "add_rmsnorm_TBps": round(3 * T * 8192 / t / 1e6, 2),
                     "silu_mul_us": round(t2, 1), "silu_mul_TBps": round(T * 28672 * 3 / t2 / 1e6, 2)})
    out["norm_act"] = rows
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
