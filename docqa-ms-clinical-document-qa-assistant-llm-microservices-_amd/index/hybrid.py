"""The semantic-indexer's IVF-PQ store (``INDEX_TYPE=ivfpq``): FAISS
``IndexRefineFlat(IndexIVFPQ)`` semantics on HBM-resident tensors.

* The exact vectors stay in a :class:`FlatIndex` (fp32, or bf16 for huge stores): they
  serve exact search until the store is large enough to train the quantizers
  (``train_min`` vectors, default 39 x nlist as FAISS recommends), and afterwards the
  refine stage -- the IVF-PQ scan (``ivfpq.hip``) proposes ``k x k_factor`` candidates
  per query and they are re-ranked with exact distances (``refine.py``), which is what
  lifts recall@10 from the PQ-quantised ordering to near exact.
* Adds go to both: the flat store and, once trained, the inverted lists (codes in HBM).
* Snapshots are FAISS files: ``IxF2`` before training, ``IxRF`` (IvPQ base + IxF2 refine
  + k_factor) after -- what ``faiss.write_index`` writes for an IndexRefineFlat.

Reference parity: the reference only has IndexFlatL2 (semantic-indexer/indexer.py:39-41);
BASELINE.json config 2 asks for the 10M-vector IVF-PQ semantic-indexer.
"""
from __future__ import annotations

import threading

import numpy as np
import torch

from . import faiss_io
from .flat import FlatIndex
from .ivfpq import IVFPQIndex
from .refine import RefineFlat


class IVFPQRefineIndex:
    def __init__(self, d: int, nlist: int = 1024, M: int = 0, nprobe: int = 32, k_factor: int = 4,
                 train_min: int = 0, device="cuda", storage_dtype=torch.float32, seed: int = 0,
                 rotation: str = "pca"):
        self.d = d
        self.metric = "l2"
        self.nlist = nlist
        self.M = M or max(1, d // 8)
        if d % self.M:
            raise ValueError(f"PQ M={self.M} must divide d={d}")
        self.nprobe = nprobe
        self.k_factor = k_factor
        self.train_min = train_min or 39 * nlist
        self.seed = seed
        self.rotation = rotation          # PQ pre-rotation (ivfpq.pca_rotation) or "none"
        self.device = torch.device(device)
        self.flat = FlatIndex(d, "l2", device, storage_dtype)
        self.ivf: IVFPQIndex | None = None
        self._lock = threading.RLock()

    # ------------------------------------------------------------------ state
    @property
    def ntotal(self) -> int:
        return self.flat.ntotal

    @property
    def trained(self) -> bool:
        return self.ivf is not None

    @property
    def xb(self) -> torch.Tensor:
        return self.flat.xb

    @property
    def norms(self) -> torch.Tensor:
        return self.flat.norms

    def _train(self) -> None:
        x = self.flat.xb.float()
        n = x.shape[0]
        cap = 256 * self.nlist                      # FAISS's max training points per centroid
        if n > cap:
            g = torch.Generator(device="cpu").manual_seed(self.seed)
            x_tr = x.index_select(0, torch.randperm(n, generator=g)[:cap].to(x.device))
        else:
            x_tr = x
        ivf = IVFPQIndex(self.d, self.nlist, self.M, 8, device=self.device, rotation=self.rotation)
        ivf.nprobe = self.nprobe
        ivf.train(x_tr, seed=self.seed)
        ivf.add(x, ids=torch.arange(n, dtype=torch.long))
        self.ivf = ivf

    # ------------------------------------------------------------------ mutation
    def add(self, x) -> None:
        x = torch.as_tensor(x)
        if x.dim() == 1:
            x = x[None]
        with self._lock:
            start = self.flat.ntotal
            self.flat.add(x)
            if self.ivf is not None:
                self.ivf.add(x.to(self.device, torch.float32),
                             ids=torch.arange(start, start + x.shape[0], dtype=torch.long))
            elif self.flat.ntotal >= self.train_min:
                self._train()

    def reset(self) -> None:
        with self._lock:
            self.flat.reset()
            self.ivf = None

    def replace(self, x, before_swap=None, ivf: IVFPQIndex | None = None) -> None:
        """Whole-content swap (index follower): the new exact vectors and (if given) an
        already-trained IVF-PQ over them, else retrain when the store is big enough."""
        with self._lock:
            self.flat.replace(x, before_swap=before_swap)
            self.ivf = ivf.to(self.device) if ivf is not None else None
            if self.ivf is None and self.flat.ntotal >= self.train_min:
                self._train()

    # ------------------------------------------------------------------ query
    def search(self, xq, k: int, id_offset: int = 0, nprobe: int | None = None):
        with self._lock:
            if self.ivf is None:
                return self.flat.search(xq, k, id_offset=id_offset)
            D, I = RefineFlat(self.ivf, self.flat.xb, "l2", self.k_factor).search(
                xq, k, nprobe=nprobe or self.nprobe)
        if id_offset:
            I = torch.where(I >= 0, I + id_offset, I)
        return D, I

    def reconstruct(self, i: int) -> np.ndarray:
        return self.flat.reconstruct(i)

    def to_numpy(self) -> np.ndarray:
        return self.flat.to_numpy()

    # ------------------------------------------------------------------ persistence
    def to_bytes(self) -> bytes:
        xb = self.flat.to_numpy()
        if self.ivf is None:
            return faiss_io.flat_bytes(xb)
        self.ivf.nprobe = self.nprobe
        return faiss_io.refine_bytes(self.ivf.to_bytes(), xb, self.k_factor)

    def save(self, path) -> None:
        with self._lock:
            faiss_io.atomic_write(path, self.to_bytes())

    @classmethod
    def from_data(cls, data, device="cuda", **kw) -> "IVFPQRefineIndex":
        """From :func:`faiss_io.read_index`'s result (flat or IxRF)."""
        if isinstance(data, faiss_io.RefineIndexData):
            base = data.base
            idx = cls(data.d, nlist=base.nlist, M=base.M, nprobe=base.nprobe,
                      k_factor=max(1, int(round(data.k_factor))), device=device, rotation=base.rotation,
                      **{k: v for k, v in kw.items() if k not in ("nlist", "M", "nprobe", "k_factor", "rotation")})
            idx.replace(torch.from_numpy(data.refine.xb), ivf=base)
            return idx
        if not isinstance(data, faiss_io.FlatIndexData):
            raise ValueError("expected a flat or IndexRefineFlat snapshot")
        idx = cls(data.d, device=device, **kw)
        if data.ntotal:
            idx.add(torch.from_numpy(data.xb))
        return idx

    @classmethod
    def load(cls, path, device="cuda", **kw) -> "IVFPQRefineIndex":
        return cls.from_data(faiss_io.read_index(path), device=device, **kw)


def make_index(settings, d: int, device) -> object:
    """The semantic-indexer's store for ``INDEX_TYPE`` (flat | ivfpq)."""
    if settings.index_type == "ivfpq":
        return IVFPQRefineIndex(d, nlist=settings.ivf_nlist, M=settings.pq_m, nprobe=settings.ivf_nprobe,
                                k_factor=settings.refine_k_factor, train_min=settings.ivf_train_min,
                                device=device, rotation=settings.pq_rotation)
    if settings.index_type != "flat":
        raise ValueError(f"INDEX_TYPE must be flat or ivfpq, got {settings.index_type!r}")
    return FlatIndex(d, "l2", device)


def load_index(settings, path, device) -> object:
    """Load a snapshot into the store type ``INDEX_TYPE`` names (an IxRF snapshot keeps its
    trained IVF-PQ; a flat snapshot under ivfpq is re-trained once large enough)."""
    data = faiss_io.read_index(path)
    if settings.index_type == "ivfpq":
        return IVFPQRefineIndex.from_data(data, device=device, nlist=settings.ivf_nlist, M=settings.pq_m,
                                          nprobe=settings.ivf_nprobe, k_factor=settings.refine_k_factor,
                                          train_min=settings.ivf_train_min, rotation=settings.pq_rotation)
    if isinstance(data, faiss_io.RefineIndexData):
        data = data.refine                           # an IVF snapshot read as exact flat
    idx = FlatIndex(data.d, "l2", device, capacity=max(1024, data.ntotal))
    if data.ntotal:
        idx.add(torch.from_numpy(data.xb))
    return idx
