"""Probe: the batch-256 gate|up projection (Llama-3-8B: N = 2 x 14336, K = 4096) as the shipped
fused-SwiGLU mid-M GEMM (mgemm cfg 2, S = 1, 224 workgroups, X re-read 224 times) against
256-wide tiles split over K into bf16 slabs (X re-read 112 times; the SwiGLU moves to a
split-K consumer).  Weights rotate over 4 copies (past the 256 MB MALL).  GPU only."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from docqa_amd import ops  # noqa: E402

assert ops.load_native()
nat = torch.ops.docqa
M, K, N = 256, 4096, 28672
x = torch.randn(M, K, device="cuda").bfloat16()
ws = [(torch.randn(N, K, device="cuda") / 64).bfloat16() for _ in range(4)]


def t(fn, it=40):
    for i in range(4):
        fn(ws[i % 4])
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(it):
        fn(ws[i % 4])
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / it


print(f"shipped mgemm_glu cfg2 S1: {t(lambda w: nat.mgemm_glu(x, w, 2)):.1f} us")
for cfg in (2, 3, 4, 6, 7):
    for S in (1, 2, 4):
        try:
            us = t(lambda w: nat.mgemm_slab16(x, w, S, cfg))
            print(f"slab16 cfg{cfg} S{S} (GEMM only): {us:.1f} us")
        except RuntimeError as e:
            print(f"slab16 cfg{cfg} S{S}: n/a")
P = nat.mgemm(x, ws[0], 2, 6)
print(f"fp32 consumer silu_mul_splitk S2: {t(lambda w: nat.silu_mul_splitk(P)):.1f} us (bf16 slabs would read half)")
