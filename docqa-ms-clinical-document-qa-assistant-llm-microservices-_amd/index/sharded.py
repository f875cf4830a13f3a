"""Vector index sharded across GPUs (one shard per data-parallel rank, 288 GB of HBM
each), searched with two collectives per query batch over RCCL/xGMI:

  1. all-gather the (padded) query batches of every rank  -> every shard answers every
     rank's queries;
  2. each rank searches its local shard (fused MFMA distance + top-k kernel) with its
     global id offset;
  3. all-gather the per-shard top-k (dist, id) pairs -- [W, nq_total, k], a few KB --
     and merge to the global top-k; every rank keeps the rows of its own queries.

Payloads are tiny (queries: nq x d fp32; results: nq x k x 12 B), so the collectives are
latency-bound and a single ring step per link is all xGMI has to carry.  Shards may be
any size (the all-gather carries explicit counts).

Reference parity: no distributed index exists in the reference (one FAISS file,
semantic-indexer/indexer.py:17-18); this is the config-5 "index sharded across 8 GPUs".
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..parallel import comm
from .flat import FlatIndex


class ShardedIndex:
    """``local``: this rank's shard -- a :class:`FlatIndex`, or any index whose
    ``search(xq, k, id_offset=..., **kw)`` returns ids (IVF-PQ: :class:`ShardedIVFPQIndex`).
    ``replicated=True``: every rank of ``group`` searches with the SAME queries (a
    tensor-parallel group serving one request stream, config 5): the query all-gather is
    skipped and each shard answers the batch once.  ``max_queries``: every rank pads its
    query batch to this static size, so no count exchange (and no host sync on the
    device counts) is needed per search; larger batches take the count-exchange path."""

    def __init__(self, local: FlatIndex, group=None, replicated: bool = False, max_queries: int | None = None):
        self.local = local
        self.group = group
        self.replicated = replicated
        self.max_queries = max_queries
        s = comm.state()
        self.world = s.dp_size if group is None else dist.get_world_size(group)
        self.rank = s.dp_rank if group is None else dist.get_rank(group)
        if group is None:
            self.group = s.dp_group
        self._offset = 0
        self._ntotal = local.ntotal
        self.refresh()

    @property
    def d(self) -> int:
        return self.local.d

    @property
    def ntotal(self) -> int:
        return self._ntotal

    def refresh(self) -> None:
        """Recompute global id offsets after local adds (collective)."""
        if self.world == 1:
            self._offset, self._ntotal = 0, self.local.ntotal
            return
        n = torch.tensor([self.local.ntotal], dtype=torch.long, device=self.local.device)
        parts = [torch.empty_like(n) for _ in range(self.world)]
        dist.all_gather(parts, n, group=self.group)
        counts = [int(p.item()) for p in parts]
        self._offset = sum(counts[: self.rank])
        self._ntotal = sum(counts)

    @property
    def id_offset(self) -> int:
        return self._offset

    def search(self, xq: torch.Tensor, k: int, **kw):
        xq = xq.to(self.local.device, dtype=torch.float32)
        if self.world == 1:
            return self.local.search(xq, k, **kw)
        nq = xq.shape[0]
        dev = xq.device
        if self.replicated:
            D, I = self.local.search(xq, k, id_offset=self._offset, **kw)
            return self._merge(D, I, k, 0, nq)
        if self.max_queries and nq <= self.max_queries:
            # static padding: the padded (zero) rows are searched too and dropped
            mx = self.max_queries
            pad = torch.zeros(mx, self.d, device=dev, dtype=torch.float32)
            pad[:nq] = xq
            allq = [torch.empty_like(pad) for _ in range(self.world)]
            dist.all_gather(allq, pad, group=self.group)
            D, I = self.local.search(torch.cat(allq, 0), k, id_offset=self._offset, **kw)
            return self._merge(D, I, k, self.rank * mx, nq)
        cnt = torch.tensor([nq], dtype=torch.long, device=dev)
        cnts = [torch.empty_like(cnt) for _ in range(self.world)]
        dist.all_gather(cnts, cnt, group=self.group)
        counts = [int(c.item()) for c in cnts]
        mx = max(counts)
        pad = torch.zeros(mx, self.d, device=dev, dtype=torch.float32)
        pad[:nq] = xq
        allq = [torch.empty_like(pad) for _ in range(self.world)]
        dist.all_gather(allq, pad, group=self.group)
        Q = torch.cat([q[:c] for q, c in zip(allq, counts)], 0)
        D, I = self.local.search(Q, k, id_offset=self._offset, **kw)
        return self._merge(D, I, k, sum(counts[: self.rank]), nq)

    def _merge(self, D, I, k: int, start: int, nq: int):
        """all-gather every shard's top-k (dist, id) and keep the global top-k of rows
        [start, start + nq)."""
        allD = [torch.empty_like(D) for _ in range(self.world)]
        allI = [torch.empty_like(I) for _ in range(self.world)]
        dist.all_gather(allD, D.contiguous(), group=self.group)
        dist.all_gather(allI, I.contiguous(), group=self.group)
        Dc = torch.cat(allD, 1)  # [tot, W*k]
        Ic = torch.cat(allI, 1)
        largest = self.local.metric == "ip"
        vals, pos = torch.topk(Dc, k, dim=1, largest=largest)
        ids = torch.gather(Ic, 1, pos)
        return vals[start:start + nq], ids[start:start + nq]


ShardedFlatIndex = ShardedIndex


class _IVFShard:
    """One rank's inverted lists (global ids stored at add time) behind the shard API."""

    metric = "l2"

    def __init__(self, ivf):
        self.ivf = ivf

    @property
    def d(self) -> int:
        return self.ivf.d

    @property
    def device(self):
        return self.ivf.device

    @property
    def ntotal(self) -> int:
        return self.ivf.ntotal

    def search(self, xq, k: int, id_offset: int = 0, nprobe: int | None = None):
        return self.ivf.search(xq, k, nprobe=nprobe)       # ids are already global


class ShardedIVFPQIndex(ShardedIndex):
    """IVF-PQ sharded across ranks (config 5 at 10M+ vectors): ONE coarse quantizer and PQ
    codebook, trained on rank 0 and broadcast, so every shard encodes into the same codes;
    each rank holds the inverted lists of its own vectors under their global ids, scans its
    lists for the probed centroids and the per-shard top-k merge is the same all-gather as
    the flat shards -- equal to one IVF-PQ over every vector."""

    @classmethod
    def build(cls, local_x, d: int, nlist: int, M: int, train_sample=None, device="cuda", group=None,
              replicated: bool = False, niter: int = 20, seed: int = 0, max_queries: int | None = None,
              rotation: str = "none"):
        from .ivfpq import IVFPQIndex

        s = comm.state()
        group = group if group is not None else s.dp_group
        rank = dist.get_rank(group) if group is not None else 0
        ivf = IVFPQIndex(d, nlist, M, 8, device=device, rotation=rotation)
        if rank == 0:
            ivf.train(train_sample, niter=niter, seed=seed)
            cent, pq = ivf.centroids.contiguous(), ivf.pq.contiguous()
            rot = ivf.rot.contiguous() if ivf.rot is not None else None
        else:
            cent = torch.empty(nlist, d, device=device)
            pq = torch.empty(M, 256, d // M, device=device)
            rot = torch.empty(d, d, device=device) if rotation != "none" else None
        if group is not None and dist.get_world_size(group) > 1:
            src = dist.get_global_rank(group, 0)
            dist.broadcast(cent, src=src, group=group)
            dist.broadcast(pq, src=src, group=group)
            if rot is not None:         # one shared pre-rotation: every shard encodes alike
                dist.broadcast(rot, src=src, group=group)
        ivf.centroids, ivf.pq, ivf.rot = cent, pq, rot
        shard = _IVFShard(ivf)
        obj = cls(shard, group=group, replicated=replicated, max_queries=max_queries)
        # global ids: this shard's offset among the ranks' vector counts
        n = int(local_x.shape[0])
        counts = torch.tensor([n], dtype=torch.long, device=device)
        if obj.world > 1:
            parts = [torch.empty_like(counts) for _ in range(obj.world)]
            dist.all_gather(parts, counts, group=obj.group)
            offs = [int(p.item()) for p in parts]
        else:
            offs = [n]
        start = sum(offs[: obj.rank])
        ivf.add(local_x, ids=torch.arange(start, start + n, dtype=torch.long))
        obj._offset, obj._ntotal = 0, sum(offs)
        return obj

    def refresh(self) -> None:   # ids are global from build time
        pass
