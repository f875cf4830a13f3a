"""Batch-1 (and few-row) decode projection sweep, timed the way the decode step runs them:
each configuration is captured into a HIP graph over `copies` distinct weight copies (rotated
past the 256 MB MALL) and replayed, so host dispatch does not count.  Reports us per call and
the effective weight-stream rate.  Usage: python scripts/b1_probe.py [M ...]"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

from docqa_amd import ops

assert ops.load_native()
nat = torch.ops.docqa


def graph_time(fn, copies, reps=20):
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
    return e0.elapsed_time(e1) * 1e3 / (reps * copies)


Ms = [int(a) for a in sys.argv[1:]] or [1]
res = []
for (name, N, K) in [("qkv", 6144, 4096), ("o", 4096, 4096), ("down", 4096, 14336), ("gate_up", 28672, 4096)]:
    nb = N * K * 2
    copies = max(2, (1 << 30) // nb + 1)
    ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(copies)]
    for M in Ms:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        if name == "gate_up":
            t = graph_time(lambda i: nat.dgemm_glu(x, ws[i]), copies)
            res.append({"proj": name, "M": M, "kind": "glu", "us": round(t, 2), "TBps": round(nb / t / 1e6, 2)})
            continue
        for tr in (64, 128):
            for S in (1, 2, 4, 7, 8, 14):
                if N % tr or K % S or (K // S) % 512:
                    continue
                t = graph_time(lambda i: nat.dgemm_partial(x, ws[i], S, tr), copies)
                res.append({"proj": name, "M": M, "tile_rows": tr, "S": S, "wgs": N // tr * S, "us": round(t, 2),
                            "TBps": round(nb / t / 1e6, 2)})
                print(json.dumps(res[-1]), flush=True)
    del ws
    torch.cuda.empty_cache()
print(json.dumps(res), flush=True)
