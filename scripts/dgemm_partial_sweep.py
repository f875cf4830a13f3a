"""Decode projection + fused split-K consumer at M = 64, per (tile rows, split) choice:
qkv -> rope_cache_splitk, o / down -> add_rmsnorm_splitk.  Weights rotate past the MALL."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

from benchmarks.bench_kernels import timeit
from docqa_amd import ops
from docqa_amd.ops import reference as R

assert ops.load_native()
nat = torch.ops.docqa
M = int(sys.argv[1]) if len(sys.argv) > 1 else 64
res = []
cs = R.rope_cos_sin(4096, 128, 500000.0, "cuda")
pos = torch.arange(M, device="cuda", dtype=torch.int32) + 600
slots = torch.arange(M, device="cuda", dtype=torch.int32) * 64
kc = torch.zeros(M + 1, 8, 64, 128, device="cuda", dtype=torch.bfloat16)
vc = torch.zeros_like(kc)
for (name, N, K) in [("qkv", 6144, 4096), ("o", 4096, 4096), ("down", 4096, 14336)]:
    nb = N * K * 2
    copies = max(2, (1 << 30) // nb + 1)
    ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(copies)]
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    g = torch.ones(N, device="cuda", dtype=torch.bfloat16)
    for tr in (64, 128):
        for S in (1, 2, 4, 7, 8, 16):
            if N % tr or K % S or (K // S) % 512:
                continue
            it = iter(range(1 << 30))
            if name == "qkv":
                fn = lambda: nat.rope_cache_splitk(nat.dgemm_partial(x, ws[next(it) % copies], S, tr), pos, cs, slots, kc, vc, 32, 8, 128)
            else:
                fn = lambda: nat.add_rmsnorm_splitk(nat.dgemm_partial(x, ws[next(it) % copies], S, tr), r, g, 1e-5)
            t = timeit(fn, iters=4 * copies)
            res.append({"proj": name, "tile_rows": tr, "S": S, "wgs": N // tr * S, "us": round(t, 1)})
    del ws
    torch.cuda.empty_cache()
print(json.dumps(res), flush=True)
