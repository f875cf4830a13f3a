"""Prefill attention probe: paged (prefix-cached) causal prefill at RAG shapes vs the
contiguous kernel, to locate the prefill-attention cost seen in the bench profile."""
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

from benchmarks.bench_kernels import timeit
from docqa_amd import ops


def main():
    assert ops.load_native()
    nat = torch.ops.docqa
    Hq, Hkv, D, BS = 32, 8, 128, 64
    scale = 1 / math.sqrt(D)
    for B, new, pre in [(128, 130, 448), (128, 130, 0), (64, 130, 448), (16, 600, 0), (128, 16, 448)]:
        W = (Hq + 2 * Hkv) * D
        T = B * new
        qkv = (torch.randn(T, W, device="cuda") * 0.5).bfloat16()
        cu = torch.arange(0, T + 1, new, device="cuda", dtype=torch.int32)
        flops = 4 * B * Hq * D * (new * pre + new * new / 2)
        if pre:
            maxb = (pre + new + BS - 1) // BS
            NB = B * maxb + 1
            kc = torch.randn(NB, Hkv, BS, D, device="cuda").bfloat16()
            vc = torch.randn_like(kc)
            bt = torch.arange(B * maxb, device="cuda", dtype=torch.int32).view(B, maxb)
            cs = torch.full((B,), pre, device="cuda", dtype=torch.int32)
            f = lambda: nat.flash_prefill_paged(qkv, cu, new, Hq, Hkv, D, scale, kc, vc, bt, cs)
        else:
            f = lambda: nat.flash_prefill(qkv, cu, new, Hq, Hkv, D, scale, True)
        t = timeit(f, iters=10)
        print(f"B={B} new={new} prefix={pre}: {t:.1f} us  {flops / t / 1e6:.1f} TFLOP/s", flush=True)
    # the bench's steady-state mix: new tokens 30..370 (mean ~90), cached prefix 320..768
    g = torch.Generator().manual_seed(0)
    B = 128
    news = (30 + torch.randint(0, 120, (B,), generator=g)).tolist()
    news[5] = 370
    pres = (64 * (5 + torch.randint(0, 8, (B,), generator=g))).tolist()
    W = (Hq + 2 * Hkv) * D
    T = sum(news)
    qkv = (torch.randn(T, W, device="cuda") * 0.5).bfloat16()
    cu = torch.tensor([0] + list(__import__("itertools").accumulate(news)), device="cuda", dtype=torch.int32)
    maxb = (max(p + n for p, n in zip(pres, news)) + BS - 1) // BS
    kc = torch.randn(B * maxb + 1, Hkv, BS, D, device="cuda").bfloat16()
    vc = torch.randn_like(kc)
    bt = torch.arange(B * maxb, device="cuda", dtype=torch.int32).view(B, maxb)
    cs = torch.tensor(pres, device="cuda", dtype=torch.int32)
    flops = sum(4 * Hq * D * (n * p + n * n / 2) for n, p in zip(news, pres))
    t = timeit(lambda: nat.flash_prefill_paged(qkv, cu, max(news), Hq, Hkv, D, scale, kc, vc, bt, cs), iters=10)
    print(f"bench-mix B={B} new mean={T / B:.0f} max={max(news)} prefix 320..768: {t:.1f} us  {flops / t / 1e6:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
