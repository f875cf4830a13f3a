"""CPU reference of the wide-probe coarse quantizer (ops.coarse_probes): ascending squared
L2 order, ties to the lower centroid id; the IVF-PQ reference search uses it."""
import torch

from docqa_amd import ops


def test_coarse_reference_order_and_ties():
    g = torch.Generator().manual_seed(0)
    cent = torch.randn(300, 32, generator=g)
    xq = torch.randn(7, 32, generator=g)
    cn = (cent ** 2).sum(1)
    p = ops.coarse_probes(xq, cent, cn, 200)
    full = ((xq[:, None, :] - cent[None]) ** 2).sum(-1)
    assert torch.equal(p, full.argsort(dim=1, stable=True)[:, :200])
    tie = torch.zeros(10, 4)
    tie[::2] = 1
    assert ops.coarse_probes(torch.zeros(1, 4), tie, (tie ** 2).sum(1), 6).tolist() == [[1, 3, 5, 7, 9, 0]]
