"""gate|up + SwiGLU at M = 256 (Llama-3-8B): unsplit mgemm cfg 2 vs the 2-way split with the
in-launch meet (cfg 6, 256-wide tiles).  Graph-timed over weight copies past the MALL.
Usage: python scripts/glu_split_probe.py [M ...]"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

from docqa_amd import ops
from docqa_amd.ops import reference as R

assert ops.load_native()
nat = torch.ops.docqa
N, K = 28672, 4096
ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(5)]
wk = ops.glu_split_workspace(512, N, "cuda")


def gt(fn, copies=5, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(copies):
            fn(i)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(copies):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / (reps * copies), 1)


for M in [int(a) for a in sys.argv[1:]] or [128, 256, 384, 512]:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    row = {"M": M, "c2": gt(lambda i: nat.mgemm_glu(x, ws[i], 2))}
    for cfg in (2, 6):
        row[f"c{cfg}_S2"] = gt(lambda i: ops.mgemm_glu_split(x, ws[i], 2, cfg, wk))
    ref = R.silu_mul((x.float() @ ws[0].float().T).bfloat16(), interleaved=True).float()
    got = ops.mgemm_glu_split(x, ws[0], 2, 6, wk).float()
    row["c6_S2_maxerr"] = round((got - ref).abs().max().item(), 4)
    print(json.dumps(row), flush=True)
