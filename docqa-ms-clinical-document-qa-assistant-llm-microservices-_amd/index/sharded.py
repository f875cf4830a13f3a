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


class ShardedFlatIndex:
    """``replicated=True``: every rank of ``group`` searches with the SAME queries (a
    tensor-parallel group serving one request stream, config 5): the query all-gather is
    skipped and each shard answers the batch once."""

    def __init__(self, local: FlatIndex, group=None, replicated: bool = False):
        self.local = local
        self.group = group
        self.replicated = replicated
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

    def search(self, xq: torch.Tensor, k: int):
        xq = xq.to(self.local.device, dtype=torch.float32)
        if self.world == 1:
            return self.local.search(xq, k)
        nq = xq.shape[0]
        dev = xq.device
        if self.replicated:
            D, I = self.local.search(xq, k, id_offset=self._offset)
            return self._merge(D, I, k, 0, nq)
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
        D, I = self.local.search(Q, k, id_offset=self._offset)
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
