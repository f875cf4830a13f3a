"""Read-side replica of the semantic-indexer's vector store for a SEPARATE process (the
llm-qa service when the services run as their own processes, `services/launch.py
--services`).

The reference's llm-qa reads ``vector_store.faiss`` + ``metadata_store.pkl`` once at import
and never sees a document indexed after it started (llm-qa/main.py:30-59, SURVEY.md §3.1
step 5).  Here the follower loads the snapshot pair and then TAILS the indexer's
write-ahead log (store/segment_log.py): every batch the indexer makes durable becomes
searchable here within one poll interval.  Every new snapshot (a new marker) is
reloaded -- it may hold rows that never went through the log (the knowledge-base
bootstrap, a startup replay) -- and the tail restarts on the rotated log after the
marker's sequence number.  Metadata is appended before vectors, so any id a concurrent
search returns has its record.
"""
from __future__ import annotations

import logging
import os
import threading
from pathlib import Path

import torch

from ..store import metadata_io
from ..store.segment_log import read_snapshot_marker, tail_frames
from . import faiss_io
from .flat import FlatIndex

log = logging.getLogger("docqa.index.follower")


class IndexFollower:
    def __init__(self, index_dir: str, index_file: str = "vector_store.faiss",
                 metadata_file: str = "metadata_store.pkl", d: int = 384, device="cuda",
                 poll_s: float = 0.2, settings=None):
        self.index_path = Path(index_dir) / index_file
        self.meta_path = Path(index_dir) / metadata_file
        self.wal_path = self.index_path.with_name(self.index_path.name + ".wal")
        self.marker_path = self.index_path.with_name(self.index_path.name + ".snapshot.json")
        # the store type the writer uses (INDEX_TYPE): flat, or IVF-PQ + exact refine
        if settings is not None:
            from .hybrid import make_index
            self.index = make_index(settings, d, device)
        else:
            self.index = FlatIndex(d, "l2", device)
        self.metadata: list[dict] = []
        self.poll_s = poll_s
        self.last_seq = 0          # highest WAL sequence applied
        self._marker = None        # snapshot marker the current state is based on
        self._offset = 0
        self._wal_ino = None
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self.version = 0

    # ------------------------------------------------------------------ load / tail
    def _load_snapshot(self) -> None:
        # the writer replaces index, metadata and marker one after the other: read the
        # marker before and after and retry until the pair is consistent
        for _ in range(20):
            mk = read_snapshot_marker(self.marker_path)
            meta = metadata_io.read_metadata(self.meta_path) if self.meta_path.exists() else []
            data = faiss_io.read_index(self.index_path) if self.index_path.exists() else None
            n = data.ntotal if data is not None else 0
            if read_snapshot_marker(self.marker_path) == mk and n == len(meta):
                break
            threading.Event().wait(0.05)
        else:
            raise RuntimeError("index snapshot kept changing under the reader")
        # the llm-qa prep thread searches this index concurrently: build the new vectors
        # off to the side and swap vectors + metadata together under the index lock, so a
        # search never sees an empty or half-loaded index (nor ids without records)
        ivf = None
        if isinstance(data, faiss_io.RefineIndexData):
            ivf, data = data.base, data.refine
        xb = torch.from_numpy(data.xb) if n else torch.empty(0, self.index.d)

        def swap_meta():
            self.metadata[:] = meta

        if ivf is not None and hasattr(self.index, "ivf"):
            self.index.replace(xb, before_swap=swap_meta, ivf=ivf)
        else:
            self.index.replace(xb, before_swap=swap_meta)
        self._marker = mk
        self.last_seq = mk["wal_seq"]
        self._offset = 0
        self.version += 1

    def poll(self) -> int:
        """Apply what the writer made durable since the last call; returns rows added."""
        if self._marker is None or read_snapshot_marker(self.marker_path) != self._marker:
            self._load_snapshot()            # first load, or the writer took a snapshot
        try:   # the writer rotates the log by replacing the file: restart at its head
            stt = os.stat(self.wal_path)
            if stt.st_ino != self._wal_ino or stt.st_size < self._offset:
                self._wal_ino, self._offset = stt.st_ino, 0
        except FileNotFoundError:
            self._offset = 0
        frames, self._offset = tail_frames(self.wal_path, self._offset)
        added = 0
        for seq, recs, vecs in frames:
            if seq <= self.last_seq:
                continue
            self.metadata.extend(recs)       # records first: every searchable id resolves
            self.index.add(torch.from_numpy(vecs.copy()))
            self.last_seq = seq
            added += len(recs)
        if added:
            self.version += 1
        return added

    # ------------------------------------------------------------------ background
    def start(self) -> "IndexFollower":
        self.poll()
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, name="index-follower", daemon=True)
            self._thread.start()
        return self

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            try:
                self.poll()
            except Exception as e:  # noqa: BLE001 - a torn read is retried next poll
                log.warning("index follower poll failed: %s", e)

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=10)
            self._thread = None
