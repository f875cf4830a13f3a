"""Exact flat vector index (IndexFlatL2 / IndexFlatIP semantics), HBM-resident.

The database lives on the GPU in a capacity-doubling buffer (``add`` is an async
device copy, amortised O(1); no host round trip), together with its fp32 squared norms
for the ``||x||^2 + ||y||^2 - 2 x.y`` decomposition.  ``search`` is one launch of the
fused MFMA distance + top-k kernel (``ops.knn``) plus its merge pass.  Storage dtype:
fp32 (exact, the FAISS format and the default) or bf16 (half the HBM bytes per scan,
for multi-million-vector shards).

Reference parity: ``faiss.IndexFlatL2(384)`` created/added at
semantic-indexer/indexer.py:39-41, written at :27, read back at llm-qa/main.py:35, and
searched with k=3 through the LangChain retriever (llm-qa/main.py:101).  Unlike the
reference, the QA side sees new vectors without a restart.
"""
from __future__ import annotations

import threading

import numpy as np
import torch

from .. import ops
from . import faiss_io


class FlatIndex:
    def __init__(self, d: int, metric: str = "l2", device="cuda", storage_dtype=torch.float32,
                 capacity: int = 1024):
        if metric not in ("l2", "ip"):
            raise ValueError("metric must be 'l2' or 'ip'")
        self.d = d
        self.metric = metric
        self.device = torch.device(device)
        self.storage_dtype = storage_dtype
        self._xb = torch.empty(capacity, d, device=self.device, dtype=storage_dtype)
        self._norms = torch.empty(capacity, device=self.device, dtype=torch.float32)
        self.ntotal = 0
        self._lock = threading.RLock()

    # ------------------------------------------------------------------ mutation
    def _grow(self, need: int) -> None:
        cap = self._xb.shape[0]
        if need <= cap:
            return
        new = max(need, cap * 2)
        xb = torch.empty(new, self.d, device=self.device, dtype=self.storage_dtype)
        nm = torch.empty(new, device=self.device, dtype=torch.float32)
        xb[: self.ntotal] = self._xb[: self.ntotal]
        nm[: self.ntotal] = self._norms[: self.ntotal]
        self._xb, self._norms = xb, nm

    def add(self, x) -> None:
        x = torch.as_tensor(x)
        if x.dim() == 1:
            x = x[None]
        if x.shape[1] != self.d:
            raise ValueError(f"dimension mismatch: {x.shape[1]} != {self.d}")
        x = x.to(self.device, dtype=torch.float32, non_blocking=True)
        with self._lock:
            n = x.shape[0]
            self._grow(self.ntotal + n)
            stored = x.to(self.storage_dtype)
            self._xb[self.ntotal:self.ntotal + n] = stored
            self._norms[self.ntotal:self.ntotal + n] = (stored.float() ** 2).sum(1)
            self.ntotal += n

    def reset(self) -> None:
        with self._lock:
            self.ntotal = 0

    def replace(self, x, before_swap=None) -> None:
        """Replace the whole content with ``x`` [n, d] without an empty or partial
        intermediate state: the new storage is built off to the side, then swapped in
        under the lock (``before_swap()``, e.g. a metadata swap, runs under the same
        lock), so a concurrent search sees either the old or the new index."""
        x = torch.as_tensor(x)
        if x.dim() == 1:
            x = x[None]
        if x.numel() and x.shape[1] != self.d:
            raise ValueError(f"dimension mismatch: {x.shape[1]} != {self.d}")
        n = x.shape[0] if x.numel() else 0
        cap = max(1024, n)
        xb = torch.empty(cap, self.d, device=self.device, dtype=self.storage_dtype)
        nm = torch.empty(cap, device=self.device, dtype=torch.float32)
        if n:
            stored = x.to(self.device, dtype=torch.float32).to(self.storage_dtype)
            xb[:n] = stored
            nm[:n] = (stored.float() ** 2).sum(1)
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        with self._lock:
            if before_swap is not None:
                before_swap()
            self._xb, self._norms, self.ntotal = xb, nm, n

    # ------------------------------------------------------------------ query
    @property
    def xb(self) -> torch.Tensor:
        return self._xb[: self.ntotal]

    @property
    def norms(self) -> torch.Tensor:
        return self._norms[: self.ntotal]

    def search(self, xq, k: int, id_offset: int = 0):
        """xq [nq, d] -> (D [nq, k] fp32, I [nq, k] int64), FAISS conventions."""
        xq = torch.as_tensor(xq)
        if xq.dim() == 1:
            xq = xq[None]
        xq = xq.to(self.device, dtype=torch.float32)
        with self._lock:
            xb, nm = self._xb, self._norms
            if xb.is_cuda:
                # the kernel may run on a side stream (the RAG prep stream) while a
                # concurrent replace()/_grow() drops these buffers: keep the caching
                # allocator from handing them out until this stream's work is done
                s = torch.cuda.current_stream(self.device)
                xb.record_stream(s)
                nm.record_stream(s)
            return ops.knn(xb[: self.ntotal], nm[: self.ntotal], xq, k, self.metric == "ip", id_offset)

    def reconstruct(self, i: int) -> np.ndarray:
        return self._xb[i].float().cpu().numpy()

    # ------------------------------------------------------------------ persistence
    def to_numpy(self) -> np.ndarray:
        return self.xb.float().cpu().numpy()

    def save(self, path) -> None:
        metric = faiss_io.METRIC_L2 if self.metric == "l2" else faiss_io.METRIC_INNER_PRODUCT
        faiss_io.write_flat(path, self.to_numpy(), metric)

    @classmethod
    def load(cls, path, device="cuda", storage_dtype=torch.float32) -> "FlatIndex":
        data = faiss_io.read_index(path)
        if not isinstance(data, faiss_io.FlatIndexData):
            raise ValueError("not a flat index")
        idx = cls(data.d, "l2" if data.metric == faiss_io.METRIC_L2 else "ip", device,
                  storage_dtype, capacity=max(1024, data.ntotal))
        if data.ntotal:
            idx.add(torch.from_numpy(data.xb))
        return idx
