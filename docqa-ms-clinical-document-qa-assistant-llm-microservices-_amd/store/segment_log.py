"""Append-only write-ahead log for the vector store.

The reference rewrites the WHOLE index + pickle after every document
(semantic-indexer/indexer.py:125, :26-30): O(N x d) bytes per message, ~30 GB per write
at the 10M x 768 config.  Here a document batch is made durable by appending ONE frame
(its metadata records + fp32 vectors, CRC-checked) to ``<index>.wal``; the FAISS /
pickle snapshot pair is rewritten only every ``snapshot_every`` batches (atomic renames)
and records the WAL sequence number it covers.  Resume = load the snapshot, replay the
frames with a higher sequence number.  A frame torn by a crash (short or CRC mismatch)
ends the replay and is truncated away, so the at-least-once redelivery of the broker
re-indexes exactly the documents whose frame never became durable.

Frame layout (little endian):
    magic  u32  'DQW1'
    seq    u64
    n      u32  vectors
    d      u32  dimension
    mlen   u32  JSON metadata bytes
    crc    u32  crc32 of (meta bytes + vector bytes)
    meta   mlen bytes   JSON list of n record dicts
    vecs   n * d * 4 bytes fp32
"""
from __future__ import annotations

import json
import os
import struct
import zlib
from pathlib import Path

import numpy as np

MAGIC = 0x31575144  # 'DQW1'
_HDR = struct.Struct("<IQIIII")


class SegmentLog:
    def __init__(self, path, fsync: bool = True):
        self.path = Path(path)
        self.fsync = fsync
        self.path.parent.mkdir(parents=True, exist_ok=True)
        self._f = None
        self.last_seq = 0
        self.bytes = 0

    # ------------------------------------------------------------------ write
    def _fh(self):
        if self._f is None:
            self._f = open(self.path, "ab")
        return self._f

    def append(self, records: list[dict], vectors: np.ndarray, seq: int | None = None) -> int:
        v = np.ascontiguousarray(vectors, dtype=np.float32)
        if v.ndim != 2 or v.shape[0] != len(records):
            raise ValueError("vectors must be [len(records), d]")
        meta = json.dumps(records, ensure_ascii=False, default=str).encode()
        body = v.tobytes()
        seq = self.last_seq + 1 if seq is None else seq
        crc = zlib.crc32(body, zlib.crc32(meta))
        f = self._fh()
        f.write(_HDR.pack(MAGIC, seq, v.shape[0], v.shape[1], len(meta), crc))
        f.write(meta)
        f.write(body)
        f.flush()
        if self.fsync:
            os.fsync(f.fileno())
        self.last_seq = seq
        self.bytes += _HDR.size + len(meta) + len(body)
        return seq

    def reset(self, seq: int) -> None:
        """Start an empty log after a snapshot covering everything up to ``seq``
        (atomic: write-then-rename, so a crash leaves either the old or the new log)."""
        self.close()
        tmp = self.path.with_suffix(self.path.suffix + ".tmp")
        with open(tmp, "wb") as f:
            f.flush()
            if self.fsync:
                os.fsync(f.fileno())
        os.replace(tmp, self.path)
        self.last_seq = seq
        self.bytes = 0

    def close(self) -> None:
        if self._f is not None:
            self._f.close()
            self._f = None

    # ------------------------------------------------------------------ read
    def replay(self, after_seq: int = 0, truncate_torn: bool = True):
        """Yield (seq, records, vectors[n, d] fp32) for every intact frame with seq >
        ``after_seq``; a torn tail is truncated (``truncate_torn``)."""
        if not self.path.exists():
            return
        good_end = 0
        with open(self.path, "rb") as f:
            while True:
                pos = f.tell()
                h = f.read(_HDR.size)
                if len(h) < _HDR.size:
                    good_end = pos if h else pos
                    break
                magic, seq, n, d, mlen, crc = _HDR.unpack(h)
                if magic != MAGIC:
                    good_end = pos
                    break
                meta = f.read(mlen)
                body = f.read(n * d * 4)
                if len(meta) < mlen or len(body) < n * d * 4 or zlib.crc32(body, zlib.crc32(meta)) != crc:
                    good_end = pos
                    break
                good_end = f.tell()
                self.last_seq = max(self.last_seq, seq)
                if seq > after_seq:
                    yield seq, json.loads(meta), np.frombuffer(body, dtype=np.float32).reshape(n, d)
        if truncate_torn and good_end < self.path.stat().st_size:
            with open(self.path, "r+b") as f:
                f.truncate(good_end)
        self.bytes = good_end


def tail_frames(path, offset: int):
    """Read intact frames from byte ``offset`` of a log another process is appending to:
    returns ([(seq, records, vectors)], new_offset).  An incomplete frame at the end (the
    writer is mid-append) is left for the next call -- never truncated here."""
    p = Path(path)
    out = []
    if not p.exists():
        return out, offset
    with open(p, "rb") as f:
        f.seek(offset)
        while True:
            h = f.read(_HDR.size)
            if len(h) < _HDR.size:
                break
            magic, seq, n, d, mlen, crc = _HDR.unpack(h)
            if magic != MAGIC:
                break
            meta = f.read(mlen)
            body = f.read(n * d * 4)
            if len(meta) < mlen or len(body) < n * d * 4 or zlib.crc32(body, zlib.crc32(meta)) != crc:
                break
            out.append((seq, json.loads(meta), np.frombuffer(body, dtype=np.float32).reshape(n, d)))
            offset = f.tell()
    return out, offset


def write_snapshot_marker(path, seq: int, ntotal: int) -> None:
    """``t`` makes every snapshot's marker distinct, so a follower notices each one."""
    import time

    tmp = Path(str(path) + ".tmp")
    tmp.write_text(json.dumps({"wal_seq": seq, "ntotal": ntotal, "t": time.time_ns()}))
    os.replace(tmp, path)


def read_snapshot_marker(path) -> dict:
    p = Path(path)
    if not p.exists():
        return {"wal_seq": 0, "ntotal": None}
    return json.loads(p.read_text())
