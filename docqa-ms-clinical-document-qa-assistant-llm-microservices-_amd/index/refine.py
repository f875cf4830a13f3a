"""Exact re-ranking of an approximate index's candidates (FAISS IndexRefineFlat semantics).

The IVF-PQ scan (csrc/kernels/ivfpq.hip) ranks by quantised distances; on embedding sets
whose nearest neighbours are nearly equidistant that ordering is noisy.  The refine stage
asks the base index for ``k * k_factor`` candidates (the scan kernel keeps up to 32 per
query) and re-ranks them with exact L2 / inner-product distances against the stored
full-precision vectors -- the same vectors a FlatIndex already keeps in HBM, shared, not
copied.  On the GPU one kernel (ivfpq.hip refine_l2_kernel: a workgroup per query, a wave
per candidate row, rank-counting top-k of <= 64) replaces the gather + einsum + topk
chain; the tensor-op path stays as the CPU implementation and the test oracle.

Reference parity: the reference only has IndexFlatL2 (semantic-indexer/indexer.py:21-22);
the 10M-vector IVF-PQ configuration is BASELINE.json config 2, where FAISS users pair
IVF-PQ with IndexRefineFlat for recall.
"""
from __future__ import annotations

import torch

from .. import ops


class RefineFlat:
    def __init__(self, base, vectors: torch.Tensor, metric: str = "l2", k_factor: int = 3):
        self.base = base
        self.xb = vectors            # [N, d] (fp32 or bf16), row i = id i
        self.metric = metric
        self.k_factor = k_factor

    @property
    def ntotal(self) -> int:
        return self.xb.shape[0]

    def search(self, xq, k: int, k_factor: int | None = None, **base_kw):
        kf = k_factor or self.k_factor
        kc = max(k, min(64, k * kf))     # the GPU top-k kernels keep up to 64 per query
        xq = torch.as_tensor(xq).to(self.xb.device, torch.float32).contiguous()
        _, cand = self.base.search(xq, kc, **base_kw)
        cand = cand.to(self.xb.device)
        if self.xb.is_cuda and self.xb.dtype in (torch.float32, torch.bfloat16) and kc <= 64:
            return ops._native().refine_flat(self.xb.contiguous(), xq, cand.contiguous(), k, self.metric == "ip")
        return self.rerank(xq, cand, k)

    def rerank(self, xq: torch.Tensor, cand: torch.Tensor, k: int):
        """Tensor-op exact re-rank (CPU path / oracle of the native kernel)."""
        kc = cand.shape[1]
        valid = cand >= 0
        rows = self.xb[cand.clamp_min(0)].float()              # [nq, kc, d]
        ip = torch.einsum("qcd,qd->qc", rows, xq)
        if self.metric == "ip":
            dist = torch.where(valid, ip, torch.full_like(ip, -float("inf")))
            D, p = torch.topk(dist, min(k, kc), dim=1, largest=True)
        else:
            dist = (rows * rows).sum(-1) - 2 * ip + (xq * xq).sum(-1, keepdim=True)
            dist = torch.where(valid, dist, torch.full_like(dist, float("inf")))
            D, p = torch.topk(dist, min(k, kc), dim=1, largest=False)
        I = torch.gather(cand, 1, p)
        bad = ~torch.isfinite(D)
        I = torch.where(bad, torch.full_like(I, -1), I)
        if k > kc:  # base returned fewer than k candidates
            pad = k - kc
            D = torch.cat([D, D.new_full((D.shape[0], pad), float("inf"))], 1)
            I = torch.cat([I, I.new_full((I.shape[0], pad), -1)], 1)
        return D, I
