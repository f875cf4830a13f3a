"""LM head + argmax at decode buckets: mgemm cfg 6 (256-wide tiles, 2-stage ring) vs cfg 8
(pgemm.hip 256 x 256 8-phase tiles with the argmax epilogue).  Graph-timed over 2 weight
copies (1 GB each: past the MALL).  Usage: python scripts/lm_cfg8_probe.py [M ...]"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

from docqa_amd import ops

assert ops.load_native()
nat = torch.ops.docqa
N, K = 128256, 4096
ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(2)]
for M in [int(a) for a in sys.argv[1:]] or [64, 128, 256, 384, 512]:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    row = {"M": M}
    for cfg in (6, 8):
        fn = lambda i: nat.mgemm_argmax(x, ws[i], N, cfg)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn(0), fn(1)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn(0), fn(1)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        row[f"cfg{cfg}_us"] = round(e0.elapsed_time(e1) * 1e3 / 20, 1)
    row["same_ids"] = bool((nat.mgemm_argmax(x, ws[0], N, 6) == nat.mgemm_argmax(x, ws[0], N, 8)).float().mean() > 0.97)
    print(json.dumps(row), flush=True)
