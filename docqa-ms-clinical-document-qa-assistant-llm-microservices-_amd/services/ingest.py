"""doc-ingestor service (FastAPI, port 8000).

Contract (doc-ingestor/main.py:19-74, processing.py:10-44):
  POST /ingest/    multipart ``file`` + ``doc_type`` (required form field)
                   -> {"message": "Ingestion réussie", "doc_id": int}
                   extraction failure -> HTTP 200 {"error": "Impossible d'extraire le texte"},
                   status ERROR_EXTRACTION; queue failure -> HTTP 200 {"error": str},
                   status ERROR_QUEUE (kept for client compatibility)
  GET  /documents/ -> all rows {id, filename, upload_date, status, doc_type}
  GET  /documents/{id} -> one row (new: readiness polling instead of a blind sleep)
  GET  /health     -> {"status": "ok", "service": "doc-ingestor"}
The raw_documents_queue message is ``{"doc_id", "text", "metadata": {"filename", "type"}}``
(key order preserved), persistent, on a durable queue.  Routes are sync ``def`` so the
blocking DB/extraction/queue work runs in the threadpool instead of stalling the event
loop as the reference's ``async def`` does.
"""
from __future__ import annotations

import datetime

import json
import os
from pathlib import Path

from fastapi import FastAPI, HTTPException, Request
from fastapi.responses import JSONResponse

from ..bus.broker import get_broker
from ..config import Settings
from ..store import docs_db
from ..text.extraction import extract_text_from_file
from ..text.dates import first_date
from .multipart import FilePart, parse_multipart


def publish_to_queue(broker, queue: str, doc_id: int, text: str, metadata: dict) -> None:
    """One persistent message on the durable ``queue`` (doc-ingestor/processing.py:21-44).

    ``broker.publish`` declares the queue, sets ``delivery_mode=2`` and, for AMQP, closes
    the connection it opened, like the reference; no channel is left open per upload."""
    body = json.dumps({"doc_id": doc_id, "text": text, "metadata": metadata})
    broker.publish(queue, body.encode())


def create_app(settings: Settings | None = None, db: docs_db.DocsDB | None = None, broker=None) -> FastAPI:
    st = settings or Settings()
    db = db or docs_db.DocsDB()
    broker = broker or get_broker(st)
    upload_dir = Path(st.upload_dir)
    upload_dir.mkdir(parents=True, exist_ok=True)
    app = FastAPI(title="DocIngestor Service (MI355X)")
    app.state.db = db
    app.state.broker = broker

    @app.post("/ingest/")
    async def ingest_document(request: Request):
        body = await request.body()
        try:
            form = parse_multipart(body, request.headers.get("content-type", ""))
        except ValueError as e:
            raise HTTPException(status_code=422, detail=str(e))
        f = form.get("file")
        doc_type = form.get("doc_type")
        if not isinstance(f, FilePart) or not isinstance(doc_type, str):
            raise HTTPException(status_code=422, detail=[{"loc": ["body", "file" if not isinstance(f, FilePart) else "doc_type"],
                                                          "msg": "field required", "type": "value_error.missing"}])
        from starlette.concurrency import run_in_threadpool

        return await run_in_threadpool(_ingest, f, doc_type)

    def _ingest(f: FilePart, doc_type: str):
        doc_id = db.create(f.filename, doc_type, docs_db.STATUS_PENDING)
        safe = os.path.basename(f.filename) or "upload"
        path = upload_dir / f"{doc_id}_{safe}"
        path.write_bytes(f.data)
        text = extract_text_from_file(str(path), st.tika_url or None)
        if not text:
            db.set_status(doc_id, docs_db.STATUS_ERROR_EXTRACTION)
            return {"error": "Impossible d'extraire le texte"}
        try:
            # the note's date (first clinical date in the raw text, else the upload day):
            # de-identification masks the dates inside the text, and the indexer's
            # patient-snippets window filter needs it (text/dates.py)
            meta = {"filename": f.filename, "type": doc_type,
                    "note_date": first_date(text) or datetime.date.today().isoformat()}
            publish_to_queue(broker, st.raw_queue, doc_id, text, meta)
            db.set_status(doc_id, docs_db.STATUS_PROCESSED)
            return {"message": "Ingestion réussie", "doc_id": doc_id}
        except Exception as e:  # noqa: BLE001 - reference returns the error text
            db.set_status(doc_id, docs_db.STATUS_ERROR_QUEUE)
            return {"error": str(e)}

    @app.get("/documents/")
    def list_documents():
        return db.list()

    @app.get("/documents/{doc_id}")
    def get_document(doc_id: int):
        d = db.get(doc_id)
        if d is None:
            return JSONResponse(status_code=404, content={"detail": "Document not found"})
        return d

    @app.get("/health")
    def health():
        return {"status": "ok", "service": "doc-ingestor"}

    return app
