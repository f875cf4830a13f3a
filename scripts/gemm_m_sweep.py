"""hipBLASLt (F.linear) time vs row count for the Llama-3-8B projections, weights rotating
past the MALL: how much do extra prefill rows cost inside a decode step's GEMMs?"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import torch.nn.functional as F

from benchmarks.bench_kernels import timeit

res = []
for (name, N, K) in [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)]:
    nb = N * K * 2
    copies = max(2, (1 << 30) // nb + 1)
    ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(copies)]
    row = {"proj": name}
    for M in (64, 128, 192, 256, 320, 512):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        it = iter(range(1 << 30))
        row[M] = round(timeit(lambda: F.linear(x, ws[next(it) % copies]), iters=4 * copies), 1)
    res.append(row)
    del ws
    torch.cuda.empty_cache()
print(json.dumps(res), flush=True)
