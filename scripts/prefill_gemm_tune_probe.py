"""Prefill GEMMs of the Llama-3-8B bench batch (M ~16k uncached prompt tokens): hipBLASLt
default heuristics vs PyTorch TunableOp's best hipBLASLt / rocBLAS solution for the same
shape.  Decides whether shipping tuned solutions for bucketed M is worth it.
Usage: python scripts/prefill_gemm_tune_probe.py [M ...]"""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import torch.nn.functional as F

from benchmarks.bench_kernels import timeit

Ms = [int(a) for a in sys.argv[1:]] or [16384]
shapes = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)]
ws = {n: (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for n, N, K in shapes}
xs = {(M, K): torch.randn(M, K, device="cuda", dtype=torch.bfloat16) for M in Ms for K in (4096, 14336)}
base = {}
for M in Ms:
    for n, N, K in shapes:
        base[(M, n)] = timeit(lambda: F.linear(xs[(M, K)], ws[n]), iters=20)
tun = torch.cuda.tunable
tun.enable(True)
tun.tuning_enable(True)
tun.set_filename(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "tunableop_probe.csv"))
for M in Ms:
    for n, N, K in shapes:
        F.linear(xs[(M, K)], ws[n])   # tunes this shape
torch.cuda.synchronize()
tun.tuning_enable(False)
for M in Ms:
    tot_b = tot_t = 0.0
    for n, N, K in shapes:
        t = timeit(lambda: F.linear(xs[(M, K)], ws[n]), iters=20)
        fl = 2 * M * N * K
        tot_b += base[(M, n)]
        tot_t += t
        print(json.dumps({"M": M, "proj": n, "default_us": round(base[(M, n)], 1), "tuned_us": round(t, 1),
                          "default_PF": round(fl / base[(M, n)] / 1e9, 3), "tuned_PF": round(fl / t / 1e9, 3)}),
              flush=True)
    print(json.dumps({"M": M, "layer_default_us": round(tot_b, 1), "layer_tuned_us": round(tot_t, 1)}), flush=True)
tun.write_file()
