"""FAISS-compatible on-disk index format (reader/writer, no faiss dependency).

Byte layout of ``faiss.write_index`` for the flat indexes, verified against the
reference's shipped ``semantic-indexer/vector_store.faiss`` (996,909 B):

    fourcc   4 B   b"IxF2" (IndexFlatL2) | b"IxFI" (IndexFlatIP)
    d        int32
    ntotal   int64
    dummy    int64 = 1 << 20
    dummy    int64 = 1 << 20
    is_trained uint8
    metric_type int32            (0 = inner product, 1 = L2)
    [metric_arg float32]         only when metric_type > 1
    n_floats uint64              = ntotal * d
    data     float32[ntotal * d] little endian

IVF-PQ (``IvPQ``) is written by :mod:`docqa_amd.index.ivfpq` with the same primitives, and
``IndexRefineFlat`` (``IxRF``: header, base index, flat refine index, float k_factor, as
faiss's index_write.cpp) wraps it for the semantic-indexer's INDEX_TYPE=ivfpq store.
No IVF fixture ships with the reference: parity with faiss for these is unpinned
(round-trip tested).
Writes are atomic (temp file + rename), fixing the reference's non-atomic
``faiss.write_index`` + ``pickle.dump`` pair (semantic-indexer/indexer.py:26-30).
"""
from __future__ import annotations

import io
import os
import struct
from dataclasses import dataclass
from pathlib import Path

import numpy as np

METRIC_INNER_PRODUCT = 0
METRIC_L2 = 1
_DUMMY = 1 << 20


@dataclass
class FlatIndexData:
    d: int
    metric: int
    xb: np.ndarray  # [ntotal, d] float32

    @property
    def ntotal(self) -> int:
        return int(self.xb.shape[0])


class Reader:
    def __init__(self, buf: bytes):
        self.b = memoryview(buf)
        self.o = 0

    def read(self, n: int) -> bytes:
        if self.o + n > len(self.b):
            raise ValueError("truncated FAISS index")
        v = bytes(self.b[self.o:self.o + n])
        self.o += n
        return v

    def unpack(self, fmt: str):
        sz = struct.calcsize(fmt)
        return struct.unpack(fmt, self.read(sz))

    def array(self, dtype, count: int) -> np.ndarray:
        nbytes = np.dtype(dtype).itemsize * count
        if self.o + nbytes > len(self.b):
            raise ValueError("truncated FAISS index payload")
        a = np.frombuffer(self.b[self.o:self.o + nbytes], dtype=dtype).copy()
        self.o += nbytes
        return a

    def vector(self, dtype) -> np.ndarray:
        (n,) = self.unpack("<Q")
        return self.array(dtype, n)


def read_header(r: Reader):
    d, = r.unpack("<i")
    ntotal, = r.unpack("<q")
    r.unpack("<qq")
    is_trained, = r.unpack("<B")
    metric, = r.unpack("<i")
    metric_arg = r.unpack("<f")[0] if metric > 1 else 0.0
    return d, ntotal, bool(is_trained), metric, metric_arg


def write_header(w: io.BufferedIOBase, d: int, ntotal: int, is_trained: bool, metric: int) -> None:
    w.write(struct.pack("<i", d))
    w.write(struct.pack("<q", ntotal))
    w.write(struct.pack("<qq", _DUMMY, _DUMMY))
    w.write(struct.pack("<B", 1 if is_trained else 0))
    w.write(struct.pack("<i", metric))


def write_vector(w, a: np.ndarray) -> None:
    a = np.ascontiguousarray(a)
    w.write(struct.pack("<Q", a.size))
    w.write(a.tobytes())


def read_flat(r: Reader, fourcc: bytes) -> FlatIndexData:
    d, ntotal, _, metric, _ = read_header(r)
    xb = r.vector(np.float32)
    if xb.size != ntotal * d:
        raise ValueError(f"flat index payload {xb.size} != {ntotal}*{d}")
    return FlatIndexData(d=d, metric=metric, xb=xb.reshape(ntotal, d))


@dataclass
class RefineIndexData:
    """``IndexRefineFlat`` (fourcc ``IxRF``): an approximate base index re-ranked with the
    exact vectors of a flat refine index."""
    base: object
    refine: FlatIndexData
    k_factor: float

    @property
    def ntotal(self) -> int:
        return self.refine.ntotal

    @property
    def d(self) -> int:
        return self.refine.d


def read_index_from(r: Reader) -> object:
    fourcc = r.read(4)
    if fourcc in (b"IxF2", b"IxFI", b"IxFl"):
        return read_flat(r, fourcc)
    if fourcc in (b"IvPQ", b"IwPQ"):
        from .ivfpq import read_ivfpq_body

        return read_ivfpq_body(r)
    if fourcc == b"IxPT":
        from .ivfpq import read_pretransform_body

        return read_pretransform_body(r)
    if fourcc == b"IxRF":
        # faiss index_write.cpp IndexRefine: header, base index, refine index, k_factor
        read_header(r)
        base = read_index_from(r)
        refine = read_index_from(r)
        k_factor, = r.unpack("<f")
        if not isinstance(refine, FlatIndexData):
            raise ValueError("IxRF: only a flat refine index is supported")
        return RefineIndexData(base, refine, float(k_factor))
    raise ValueError(f"unsupported FAISS index type {fourcc!r}")


def read_index(path) -> object:
    return read_index_from(Reader(Path(path).read_bytes()))


def refine_bytes(base_bytes: bytes, xb: np.ndarray, k_factor: float, metric: int = METRIC_L2) -> bytes:
    """IndexRefineFlat(base) with the exact vectors ``xb`` as its refine index."""
    w = io.BytesIO()
    w.write(b"IxRF")
    write_header(w, int(xb.shape[1]) if xb.ndim == 2 else 0, int(xb.shape[0]), True, metric)
    w.write(base_bytes)
    w.write(flat_bytes(xb, metric))
    w.write(struct.pack("<f", float(k_factor)))
    return w.getvalue()


def flat_bytes(xb: np.ndarray, metric: int = METRIC_L2) -> bytes:
    xb = np.ascontiguousarray(xb, dtype=np.float32)
    n, d = xb.shape if xb.ndim == 2 else (0, 0)
    w = io.BytesIO()
    w.write(b"IxF2" if metric == METRIC_L2 else b"IxFI")
    write_header(w, d, n, True, metric)
    write_vector(w, xb.reshape(-1))
    return w.getvalue()


def atomic_write(path, data: bytes) -> None:
    path = Path(path)
    tmp = path.with_name(f".{path.name}.tmp.{os.getpid()}")
    with open(tmp, "wb") as f:
        f.write(data)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def write_flat(path, xb: np.ndarray, metric: int = METRIC_L2) -> None:
    atomic_write(path, flat_bytes(xb, metric))
