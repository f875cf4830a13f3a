"""k-means for IVF coarse quantizers and PQ codebooks, on the GPU.

Assignment of each training point to its nearest centroid is the flat kNN kernel with
k=1 (MFMA distance tile + fused arg-min) -- the same kernel that serves search; the
update is an ``index_add_`` scatter of the points into per-centroid sums.  Empty
clusters are re-seeded by splitting the largest one (FAISS's policy).  Training samples
``max_points_per_centroid * k`` points (FAISS default 256).
"""
from __future__ import annotations

import torch

from .. import ops


def assign(x: torch.Tensor, centroids: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    d = x.shape[1]
    if d % 8:  # the MFMA kernel wants d % 8 == 0: zero columns leave distances unchanged
        pad = 8 - d % 8
        x = torch.nn.functional.pad(x.float(), (0, pad))
        centroids = torch.nn.functional.pad(centroids.float(), (0, pad))
    norms = (centroids.float() ** 2).sum(1)
    D, I = ops.knn(centroids.float().contiguous(), norms, x.float().contiguous(), 1, False, 0)
    return D[:, 0], I[:, 0]


def kmeans(x: torch.Tensor, k: int, niter: int = 20, seed: int = 0,
           max_points_per_centroid: int = 256) -> torch.Tensor:
    """x [n, d] fp32 -> centroids [k, d] fp32 (on x's device)."""
    n, d = x.shape
    g = torch.Generator(device="cpu").manual_seed(seed)
    if n > k * max_points_per_centroid:
        sel = torch.randperm(n, generator=g)[: k * max_points_per_centroid].to(x.device)
        x = x.index_select(0, sel)
        n = x.shape[0]
    if n < k:
        raise ValueError(f"need at least {k} training points, got {n}")
    x = x.float().contiguous()
    cent = x.index_select(0, torch.randperm(n, generator=g)[:k].to(x.device)).clone()
    for _ in range(niter):
        _, a = assign(x, cent)
        sums = torch.zeros_like(cent).index_add_(0, a, x)
        cnt = torch.zeros(k, device=x.device, dtype=torch.float32).index_add_(
            0, a, torch.ones(n, device=x.device))
        empty = cnt == 0
        cent = torch.where(empty[:, None], cent, sums / cnt.clamp(min=1)[:, None])
        if bool(empty.any()):
            big = int(cnt.argmax())
            for e in torch.nonzero(empty).flatten().tolist():
                eps = 1e-4 * torch.randn(d, generator=g).to(x.device)
                cent[e] = cent[big] + eps
                cent[big] = cent[big] - eps
    return cent


def kmeans_subspaces(x: torch.Tensor, M: int, ksub: int = 256, niter: int = 15, seed: int = 0) -> torch.Tensor:
    """PQ codebook training: independent k-means per sub-space -> [M, ksub, d/M]."""
    n, d = x.shape
    dsub = d // M
    books = []
    for m in range(M):
        books.append(kmeans(x[:, m * dsub:(m + 1) * dsub].contiguous(), ksub, niter, seed + m))
    return torch.stack(books)
