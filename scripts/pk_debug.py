import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
from docqa_amd import ops
ops.load_native()
nat = torch.ops.docqa
torch.manual_seed(0)
for (N, K, S) in [(256, 64, 1), (256, 128, 1), (256, 256, 1), (512, 128, 1), (256, 128, 2)]:
    x = torch.randn(256, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    ref = x.float() @ w.float().T
    got = nat.wgemm(x, ops.pack_fragments(w), S, 17)
    got = got.float() if S == 1 else got.sum(0)
    bad = (got - ref).abs() > 0.05 * ref.abs().max()
    cols = bad.any(0).nonzero().flatten().tolist()
    rows = bad.any(1).nonzero().flatten().tolist()
    print(N, K, S, "bad cols", len(cols), cols[:20], "bad rows", len(rows), rows[:10])
    if cols:
        c = cols[0]
        # which W row matches the computed column?
        sims = ((x.float() @ w.float().T) - got[:, c:c+1]).abs().max(0).values
        print("  col", c, "best matching W row", int(sims.argmin()), float(sims.min()))
