"""Vector index sharded across GPUs (one shard per data-parallel rank, 288 GB of HBM
each), searched with two collectives per query batch over RCCL/xGMI:

  1. all-gather the (padded) query batches of every rank  -> every shard answers every
     rank's queries;
  2. each rank searches its local shard (fused MFMA distance + top-k kernel) with its
     global id offset;
  3. all-gather the per-shard top-k (dist, id) pairs -- [W, nq_total, k], a few KB --
     and merge to the global top-k; every rank keeps the rows of its own queries.

Payloads are tiny (queries: nq x d fp32; results: nq x k x 12 B), so the collectives are
latency-bound.  On the GPU both all-gathers run on the IPC peer-memory kernel
(parallel/custom_ar.py GATHER mode: every rank reads its peers' staging buffers over all
xGMI links at once, graph-capturable, off RCCL) when ``enable_ipc`` succeeded; RCCL /
gloo ``all_gather`` is the fallback (CPU, or a node without IPC).  Shards may be any size
(the count-exchange path carries explicit counts).

Failure surfacing: the IPC gather gives up on a peer after a bounded wait and records it
in a sticky error word instead of hanging the GPU; its results are then stale.  Every
search through the IPC path snapshots that word behind its kernels (no extra sync) and
``check_gather()`` -- called by the pipeline right after its existing host sync on the
hits -- raises :class:`CollectiveError`, so a late or dead rank can never turn into
silently wrong retrieval.  Data-parallel ranks are not in lockstep (EOS-dependent batch
lengths, the pipelined lead, first-call setup), so the shard gathers wait up to
``DOCQA_SHARD_GATHER_TIMEOUT_MS`` (default 60 s) rather than the TP all-reduce's 500 ms.

Reference parity: no distributed index exists in the reference (one FAISS file,
semantic-indexer/indexer.py:17-18); this is the config-5 "index sharded across 8 GPUs".
"""
from __future__ import annotations

import threading

import os

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
        self._ipc = None
        self.ipc_status = "process-group gather"   # enable_ipc: "ipc" once its handshake passed
        # per-thread search state: the error-word snapshot of this thread's last IPC search
        # (a serving front end searches from its prep thread while the indexer searches from
        # request threads; one instance-wide slot let one thread's search overwrite
        # another's snapshot before it was checked -- ADVICE r5)
        self._tls = threading.local()
        self.refresh()

    def enable_ipc(self, max_bytes: int = 16 << 20, factory=None) -> bool:
        """Route the per-batch all-gathers through the IPC peer-memory kernel (collective:
        every rank of the group calls it; all fall back to RCCL together if the kernel cannot
        be set up).  Once set up, a handshake gather (:meth:`_handshake`) must return every
        peer's row exactly, else the run fails with :class:`CollectiveError` before the
        first search.  ``factory``: the gather's constructor (tests)."""
        if self.world == 1 or self._ipc is not None or self.local.device.type != "cuda":
            return self._ipc is not None
        from ..parallel.custom_ar import CollectiveError

        if factory is None:
            from ..parallel.custom_ar import CustomAllReduce as factory

        timeout_ms = float(os.environ.get("DOCQA_SHARD_GATHER_TIMEOUT_MS", "60000"))
        try:
            self._ipc = factory(group=self.group, max_bytes=max_bytes, device=self.local.device,
                                timeout_ms=timeout_ms)
        except Exception as e:  # noqa: BLE001 - collective decision inside the constructor
            print(f"[sharded] IPC all-gather unavailable ({e}); using the process group", flush=True)
            self._ipc = None
            self.ipc_status = "unavailable: process-group gather"
        if self._ipc is not None:
            try:
                self._handshake()
            except CollectiveError as e:
                # DOCQA_IPC_HANDSHAKE=strict: fail the run here.  Default (fallback): every
                # rank saw the same verdict (_handshake agrees over the process group), so all
                # of them drop the IPC path together and gather through the process group --
                # never a silently wrong merge; bench.py's sharded-vs-unsharded check still
                # runs at the end, and ipc_status says what happened
                if os.environ.get("DOCQA_IPC_HANDSHAKE", "fallback") == "strict":
                    raise
                print(f"[sharded] {e}; falling back to the process-group gather", flush=True)
                try:
                    self._ipc.close()
                except Exception:  # noqa: BLE001 - best effort, the path is abandoned either way
                    pass
                self._ipc = None
                self.ipc_status = "handshake failed: process-group gather"
                return False
            self.ipc_status = "ipc"
        return self._ipc is not None

    def _handshake(self) -> None:
        """One gather through the IPC path of a row every rank can predict for every peer --
        (rank, world, shard offset, shard size, magic) -- checked word for word: a peer
        mapping that reads the wrong buffer, a stale staging row or a rank that never
        arrives fails the run here (all ranks agree on the outcome over the process group),
        not as silently wrong top-k later.  The offsets / sizes come from :meth:`refresh`'s
        process-group exchange, independent of the IPC path.  Reference: the k = 3 retrieval
        of llm-qa/main.py:101, which must not silently change."""
        from ..parallel.custom_ar import CollectiveError, _agree

        magic = 0x5D0C0A11
        sizes = self._shard_sizes()
        offs = [sum(sizes[:r]) for r in range(self.world)]

        def row(r: int) -> list[int]:
            return [r, self.world, offs[r], sizes[r], magic, r ^ magic, 0, 0]

        dev = getattr(self._ipc, "device", self.local.device)
        mine = torch.tensor(row(self.rank), dtype=torch.int32, device=dev)
        got = self._ipc.all_gather_raw(mine).view(self.world, -1).cpu()
        want = torch.tensor([row(r) for r in range(self.world)], dtype=torch.int32)
        ok = bool(torch.equal(got, want))
        try:
            self._ipc.check()
        except Exception:  # noqa: BLE001 - a peer that never arrived
            ok = False
        if dist.is_initialized():
            ok = _agree(ok, self.group, dev)
        if not ok:
            bad = [r for r in range(self.world) if not torch.equal(got[r], want[r])]
            raise CollectiveError(f"sharded index: IPC handshake gather returned wrong peer rows "
                                  f"{bad or '(on another rank)'}; refusing to serve sharded retrieval")

    def _shard_sizes(self) -> list[int]:
        """Every rank's shard size (the counts :meth:`refresh` exchanged)."""
        sizes = getattr(self, "_sizes", None)
        if sizes is None or len(sizes) != self.world:
            raise RuntimeError("shard sizes unknown: call refresh() first")
        return list(sizes)

    def _all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape] -- IPC peer-memory gather when enabled, else the process group."""
        t = t.contiguous()
        if self._ipc is not None and t.is_cuda:
            nb = t.numel() * t.element_size()
            if nb % 16 == 0 and nb // 2 <= self._ipc.max_elems:
                self._tls.used_ipc = True
                return self._ipc.all_gather_raw(t)
        parts = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t, group=self.group)
        return torch.stack(parts)

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
            self._sizes = [self.local.ntotal]
            return
        n = torch.tensor([self.local.ntotal], dtype=torch.long, device=self.local.device)
        parts = [torch.empty_like(n) for _ in range(self.world)]
        dist.all_gather(parts, n, group=self.group)
        counts = [int(p.item()) for p in parts]
        self._sizes = counts
        self._offset = sum(counts[: self.rank])
        self._ntotal = sum(counts)

    @property
    def id_offset(self) -> int:
        return self._offset

    def check_gather(self) -> None:
        """Raise :class:`~docqa_amd.parallel.custom_ar.CollectiveError` if a peer never
        arrived at the last search's IPC gathers.  Call after a host sync that covers the
        search (e.g. ``I.tolist()`` on the search's stream): the snapshot copy was queued
        behind the gathers, so it is complete by then and reading it costs nothing."""
        snap = getattr(self._tls, "snap", None)
        self._tls.snap = None
        if snap is not None and self._ipc is not None:
            self._ipc.raise_if(snap)

    def search(self, xq: torch.Tensor, k: int, **kw):
        xq = xq.to(self.local.device, dtype=torch.float32)
        if self.world == 1:
            return self.local.search(xq, k, **kw)
        self._tls.used_ipc = False
        D, I = self._search(xq, k, **kw)
        if self._tls.used_ipc:
            # stream-ordered copy of the sticky error word behind this search's gathers
            # (this thread's: check_gather() of the same thread reads it)
            self._tls.snap = self._ipc.snapshot()
        return D, I

    def _search(self, xq: torch.Tensor, k: int, **kw):
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
            allq = self._all_gather(pad)
            D, I = self.local.search(allq.view(self.world * mx, self.d), k, id_offset=self._offset, **kw)
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
        rows = D.shape[0]
        # one payload per batch: fp32 distances and int64 ids side by side as int32 words
        pack = torch.cat([D.float().contiguous().view(torch.int32), I.to(torch.int64).contiguous().view(torch.int32)], 1)
        if (pack.numel() * 4) % 16:
            pad = torch.zeros(4 - pack.numel() % 4, dtype=torch.int32, device=pack.device)
            flat = torch.cat([pack.view(-1), pad])
            allp = self._all_gather(flat)[:, : pack.numel()].reshape(self.world, rows, 3 * k)
        else:
            allp = self._all_gather(pack)
        allD = allp[:, :, :k].contiguous().view(torch.float32)               # [W, rows, k]
        allI = allp[:, :, k:].contiguous().view(torch.int64)
        Dc = allD.permute(1, 0, 2).reshape(rows, self.world * k)   # [tot, W*k]
        Ic = allI.permute(1, 0, 2).reshape(rows, self.world * k)
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
        obj._sizes = offs
        return obj

    def refresh(self) -> None:   # ids are global from build time
        pass
