"""Locate dgemm mismatches: per (shape, M, S) report max error and where it sits."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

from docqa_amd import ops

assert ops.load_native()
torch.manual_seed(0)
for (N, K) in [(28672, 4096), (4096, 4096), (1024, 4096), (256, 4096), (64, 512), (64, 4096)]:
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    for M in (1, 16, 64):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        ref = x.float() @ w.float().T
        for S in (1, 2):
            if (K // S) % 128:
                continue
            errs = []
            for rep in range(3):
                o = torch.ops.docqa.dgemm(x, w, S).float()
                e = (o - ref).abs()
                errs.append(round(e.max().item(), 3))
            bad = (e > 0.05).nonzero()
            where = ""
            if len(bad):
                rows = bad[:, 0].unique().tolist()[:8]
                cols = bad[:, 1].unique()
                where = f"bad={len(bad)} rows={rows} cols[{cols.min().item()}..{cols.max().item()}] ncols={len(cols)} tiles={sorted(set((cols // 64).tolist()))[:10]}"
            print(N, K, M, S, errs, where, flush=True)
