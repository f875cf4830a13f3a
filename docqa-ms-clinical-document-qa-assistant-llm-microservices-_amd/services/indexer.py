"""semantic-indexer service: clean_documents_queue consumer + search HTTP API (port 8003).

Reference (semantic-indexer/indexer.py:11-143):
  * startup: load ``vector_store.faiss`` + ``metadata_store.pkl`` if both exist (resume),
    else build from the ``default_data`` CSVs and save;
  * consume clean documents (prefetch 1): ``text[i:i+500]`` chunks labelled
    ``"Dossier Patient {doc_id}"`` / ``"patient_file"``, add, save, ack;
  * ``add_to_index`` skips blank text.
Fixes, each covered by tests: the whole document is embedded in one packed GPU batch
instead of one encode per chunk; a batch is made durable by one append to a CRC-framed
write-ahead log (store/segment_log.py) and acked, the full snapshot pair is rewritten
only every ``INDEX_SNAPSHOT_EVERY`` batches (the reference rewrites O(N x d) bytes per
document), resume = snapshot + WAL replay; snapshots are atomic (temp + rename, index
before metadata) so a reader never sees mismatched lengths; one writer lock serialises index
mutation (multiple consumers are safe); the QA side shares the live index object in
process (no restart needed to see new documents); metadata ``doc_id`` is the real
document id.
HTTP (the endpoint the reference's synthese-comparative expects but nobody served,
synthese-comparative/core/retrieval_client.py:72-91):
  GET  /api/search/patient-snippets?patient_id&from_date&to_date&focus -> [{doc_id, text}]
  POST /api/search {"query", "k"} -> hits;  GET /api/index/stats;  GET /health
"""
from __future__ import annotations

import json
import logging
import threading
import time
from pathlib import Path

import torch
from fastapi import FastAPI
from fastapi.responses import JSONResponse

from ..bus.broker import get_broker
from ..config import Settings
from ..index import faiss_io
from ..index.flat import FlatIndex  # noqa: F401  (the default store type)
from ..index.hybrid import load_index, make_index
from ..pipeline.corpus import embed_records
from ..schemas import SearchRequest
from ..store import metadata_io
from ..store.segment_log import SegmentLog, read_snapshot_marker, write_snapshot_marker
from ..text.chunking import chunk_chars
from ..text.dates import in_window, parse_date
from ..utils import tracing
from ..text.kb import kb_records_from_dir, synthetic_kb_records

logger = logging.getLogger("semantic-indexer")


class PatientIndex:
    """patient key -> its patient-file row ids, kept beside the append-only metadata list.

    ``/api/search/patient-snippets`` (the contract of synthese-comparative/core/
    retrieval_client.py:72-91) used to scan every metadata row under the index lock; at the
    10M-chunk scale of config 2 that stalls every search for seconds.  The map is updated
    by every ``add_records`` / WAL replay and rebuilt once from a loaded snapshot, so a
    lookup costs O(rows of that patient).  A row is reachable by its ``patient_id`` and by
    its ``doc_id`` (the reference keys patient chunks by document id)."""

    def __init__(self):
        self._rows: dict[str, list[int]] = {}
        self.n = 0          # metadata rows covered so far

    def extend(self, metadata: list[dict], start: int | None = None) -> None:
        start = self.n if start is None else start
        for i in range(start, len(metadata)):
            m = metadata[i]
            if m.get("type") != "patient_file":
                continue
            keys = {str(m.get("patient_id")), str(m.get("doc_id"))}
            for k in keys:
                self._rows.setdefault(k, []).append(i)
        self.n = max(self.n, len(metadata))

    def rebuild(self, metadata: list[dict]) -> None:
        self._rows, self.n = {}, 0
        self.extend(metadata, 0)

    def rows(self, key: str) -> list[int]:
        return list(self._rows.get(str(key), ()))


class SemanticIndexer:
    def __init__(self, encoder, tokenizer, settings: Settings | None = None, index: FlatIndex | None = None,
                 metadata: list | None = None, device: str = "cuda", on_indexed=None):
        self.st = settings or Settings()
        self.encoder = encoder
        self.tok = tokenizer
        self.device = device
        self.index = index
        self.metadata: list[dict] = metadata if metadata is not None else []
        self.patients = PatientIndex()
        self.patients.rebuild(self.metadata)
        self.lock = threading.RLock()
        self.on_indexed = on_indexed  # callback(doc_id) e.g. docs DB status -> INDEXED
        self._ch = None
        self._depth = None          # broker queue-depth probe (group commit), None: per message
        self._pending: list = []
        self.version = 0
        self.wal = SegmentLog(self.index_path.with_name(self.index_path.name + ".wal")) if self.st.index_wal else None
        self._batches_since_snapshot = 0

    # ------------------------------------------------------------------ paths
    @property
    def index_path(self) -> Path:
        return Path(self.st.index_dir) / self.st.index_file

    @property
    def meta_path(self) -> Path:
        return Path(self.st.index_dir) / self.st.metadata_file

    # ------------------------------------------------------------------ lifecycle
    @property
    def marker_path(self) -> Path:
        return self.index_path.with_name(self.index_path.name + ".snapshot.json")

    def startup(self, build_if_missing: bool = True) -> "SemanticIndexer":
        with self.lock:
            dirty = False
            covered = 0
            if self.index_path.exists() and self.meta_path.exists():
                self.index = load_index(self.st, self.index_path, self.device)
                self.metadata = metadata_io.read_metadata(self.meta_path)
                self.patients.rebuild(self.metadata)
                if len(self.metadata) != self.index.ntotal:
                    raise RuntimeError(f"index/metadata mismatch: {self.index.ntotal} vs {len(self.metadata)}")
                covered = read_snapshot_marker(self.marker_path)["wal_seq"]
                logger.info("resumed index (%d vectors)", self.index.ntotal)
            else:
                self.index = make_index(self.st, self.encoder.cfg.hidden, self.device)
                self.metadata = []
                self.patients.rebuild(self.metadata)
                if build_if_missing:
                    recs = kb_records_from_dir(self.st.default_data_dir) or synthetic_kb_records()
                    self.add_records(recs, log=False)
                    dirty = True
            if self.wal is not None:   # batches made durable after the last snapshot
                replayed = 0
                for _, recs, vecs in self.wal.replay(after_seq=covered):
                    self.index.add(torch.from_numpy(vecs.copy()))
                    self.metadata.extend(recs)
                    self.patients.extend(self.metadata)
                    replayed += len(recs)
                if replayed:
                    logger.info("replayed %d vectors from the write-ahead log", replayed)
                    self.version += 1
                    dirty = True
            if dirty:
                self.save_state()
        return self

    def save_state(self) -> None:
        with self.lock:
            Path(self.st.index_dir).mkdir(parents=True, exist_ok=True)
            self.index.save(self.index_path)            # atomic
            metadata_io.write_metadata(self.meta_path, self.metadata)  # atomic
            if self.wal is not None:                    # snapshot covers the whole log
                seq = self.wal.last_seq
                write_snapshot_marker(self.marker_path, seq, self.index.ntotal)
                self.wal.reset(seq)
            self._batches_since_snapshot = 0

    def commit(self) -> None:
        """Make the batches indexed so far durable: a WAL append already did; take a
        full snapshot every ``snapshot_every`` batches (always, without a WAL)."""
        self._batches_since_snapshot += 1
        if self.wal is None or self._batches_since_snapshot >= self.st.snapshot_every:
            self.save_state()

    # ------------------------------------------------------------------ mutation
    def add_records(self, records: list[dict], log: bool = True) -> int:
        recs = [r for r in records if r.get("text_content", "").strip()]
        if not recs:
            return 0
        with tracing.span("indexer.embed", chunks=len(recs)):
            emb = embed_records(self.encoder, self.tok, recs)
        with self.lock:
            if self.index is None:
                self.index = make_index(self.st, self.encoder.cfg.hidden, self.device)
            if log and self.wal is not None:           # durable before it is visible
                self.wal.append(recs, emb.float().cpu().numpy())
            self.index.add(emb)
            self.metadata.extend(recs)
            self.patients.extend(self.metadata)
            self.version += 1
        return len(recs)

    def add_to_index(self, text: str, source_name: str, doc_type: str = "knowledge_base", doc_id: str = "KB") -> bool:
        """Reference-compatible single add (blank text skipped)."""
        return self.add_records([{"doc_id": doc_id, "text_content": text, "source": source_name,
                                  "type": doc_type}]) == 1

    def index_document(self, doc_id, text: str, metadata: dict | None = None) -> int:
        md = metadata or {}
        recs = [{"doc_id": str(doc_id), "text_content": c, "source": f"Dossier Patient {doc_id}",
                 "type": "patient_file", "patient_id": md.get("patient_id", str(doc_id)),
                 "filename": md.get("filename"), "note_date": parse_date(md.get("note_date"))}
                for c in chunk_chars(text or "", self.st.chunk_size)]
        return self.add_records(recs)

    # ------------------------------------------------------------------ queue
    def callback(self, ch, method, properties, body):
        """Queue consumer (reference semantics: chunk, embed, persist, then ack).

        Adaptive group commit: while more clean documents are already waiting in the
        queue (up to ``BATCH_DOCS``), messages are only collected; the batch is then
        embedded in one packed encoder forward, persisted with ONE atomic snapshot and
        acked together.  An idle queue flushes at once, so single-document latency is
        unchanged; a burst no longer pays one index snapshot per document."""
        self._pending.append((ch, method, body))
        waiting = self._depth(self.st.clean_queue) if self._depth is not None else 0
        if waiting > 0 and len(self._pending) < self.BATCH_DOCS:
            return
        batch, self._pending = self._pending, []
        recs, done = [], []
        for c, m, b in batch:
            try:
                msg = json.loads(b)
                doc_id = msg.get("doc_id")
                md = msg.get("metadata") or {}
                recs.extend({"doc_id": str(doc_id), "text_content": chunk, "source": f"Dossier Patient {doc_id}",
                             "type": "patient_file", "patient_id": md.get("patient_id", str(doc_id)),
                             "filename": md.get("filename"), "note_date": parse_date(md.get("note_date"))}
                            for chunk in chunk_chars(msg.get("original_text_masked", "") or "", self.st.chunk_size))
                done.append((c, m, doc_id))
            except Exception as e:  # noqa: BLE001 - malformed message: dead-letter it
                logger.error("indexing error: %s", e)
                c.basic_nack(delivery_tag=m.delivery_tag, requeue=False)
        try:
            n = self.add_records(recs)
            self.commit()
        except Exception as e:  # noqa: BLE001
            logger.error("indexing error: %s", e)
            for c, m, _ in done:
                c.basic_nack(delivery_tag=m.delivery_tag, requeue=False)
            return
        for c, m, doc_id in done:
            c.basic_ack(delivery_tag=m.delivery_tag)
            if self.on_indexed is not None and isinstance(doc_id, int):
                self.on_indexed(doc_id)
        logger.info("indexed %d doc(s) (%d chunks)", len(done), n)

    BATCH_DOCS = 64

    def start_consumer(self, broker=None) -> threading.Thread:
        broker = broker or get_broker(self.st)
        ch = broker.channel()
        self._ch = ch
        self._depth = getattr(broker, "depth", None)
        ch.queue_declare(queue=self.st.clean_queue, durable=True)
        ch.basic_qos(prefetch_count=self.BATCH_DOCS if self._depth is not None else 1)
        ch.basic_consume(queue=self.st.clean_queue, on_message_callback=self.callback)
        t = threading.Thread(target=ch.start_consuming, name="indexer-consumer", daemon=True)
        t.start()
        return t

    def stop_consumer(self) -> None:
        if self._ch is not None:
            self._ch.stop_consuming()

    # ------------------------------------------------------------------ query
    @torch.inference_mode()
    def search(self, query: str, k: int = 3) -> list[dict]:
        q = self.encoder.encode(self.tok.encode_batch([query]))
        with self.lock:
            D, I = self.index.search(q, k)
            dl, il = D[0].tolist(), I[0].tolist()
            # a sharded index: surface a failed cross-rank gather (stale peer rows) after the
            # host sync above instead of serving it (index/sharded.py check_gather)
            check = getattr(self.index, "check_gather", None)
            if check is not None:
                check()
            out = []
            for d, i in zip(dl, il):
                if 0 <= i < len(self.metadata):
                    m = self.metadata[i]
                    out.append({"id": i, "score": d, "text": m.get("text_content", ""), "source": m.get("source"),
                                "type": m.get("type"), "doc_id": str(m.get("doc_id"))})
            return out

    def patient_snippets(self, patient_id: str, from_date=None, to_date=None, focus=None, limit: int = 20) -> list[dict]:
        """The patient's chunks, optionally restricted to notes dated in [from_date, to_date]
        (each chunk's ``note_date``, set at ingest: text/dates.py) and ranked by distance to
        the ``focus`` text."""
        pid = str(patient_id)
        lo, hi = parse_date(from_date), parse_date(to_date)
        with self.lock:   # O(rows of this patient): the per-patient map, never a metadata scan
            ids = self.patients.rows(pid)
            meta = self.metadata
        rows = [(i, meta[i]) for i in ids if in_window(meta[i].get("note_date"), lo, hi)]
        if focus and rows:
            q = self.encoder.encode(self.tok.encode_batch([focus]))
            ids = torch.tensor([i for i, _ in rows], device=self.index.xb.device)
            with self.lock:
                xb = self.index.xb.index_select(0, ids).float()
            d = ((xb - q.to(xb.device)) ** 2).sum(1)
            order = d.argsort().tolist()
            rows = [rows[j] for j in order]
        return [{"doc_id": str(m.get("doc_id")), "text": m.get("text_content", "")} for _, m in rows[:limit]]


def create_app(indexer: SemanticIndexer) -> FastAPI:
    app = FastAPI(title="Semantic Indexer (MI355X)")
    app.state.indexer = indexer

    @app.get("/health")
    def health():
        return {"status": "ok", "service": "semantic-indexer"}

    @app.get("/debug/trace")
    def trace_dump():
        return tracing.chrome_trace()

    @app.get("/api/index/stats")
    def stats():
        idx = indexer.index
        return {"ntotal": idx.ntotal if idx is not None else 0, "dim": idx.d if idx is not None else None,
                "metric": idx.metric if idx is not None else None, "version": indexer.version}

    @app.post("/api/search")
    def search(req: SearchRequest):
        if indexer.index is None:
            return JSONResponse(status_code=503, content={"detail": "Index non chargé."})
        return indexer.search(req.query, req.k)

    @app.get("/api/search/patient-snippets")
    def patient_snippets(patient_id: str, from_date: str | None = None, to_date: str | None = None,
                         focus: str | None = None):
        return indexer.patient_snippets(patient_id, from_date, to_date, focus)

    return app
