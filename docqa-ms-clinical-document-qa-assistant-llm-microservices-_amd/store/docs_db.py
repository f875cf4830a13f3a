"""Document-metadata store of the doc-ingestor (SQLAlchemy).

Schema identical to the reference's ``documents`` table (doc-ingestor/models.py:5-12):
``id SERIAL PK, filename, upload_date timestamptz default now(), status, doc_type``.
Status lifecycle: PENDING -> PROCESSED | ERROR_EXTRACTION | ERROR_QUEUE
(doc-ingestor/main.py:28,44,54,63), extended with INDEXED once the semantic indexer has
made the document searchable (the reference has no readiness signal: its UI sleeps 5 s,
clinical-ui/app.py:55-58).

Backend: ``DATABASE_URL`` (default SQLite file); ``DOCQA_DB=postgres`` builds the
reference URL ``postgresql://admin:adminpassword@DB_HOST:DB_PORT/ingestion_db``
(doc-ingestor/database.py:10).
"""
from __future__ import annotations

import os
import threading

from sqlalchemy import Column, DateTime, Integer, String, create_engine
from sqlalchemy.orm import declarative_base, sessionmaker
from sqlalchemy.pool import StaticPool
from sqlalchemy.sql import func

Base = declarative_base()

STATUS_PENDING = "PENDING"
STATUS_PROCESSED = "PROCESSED"
STATUS_ERROR_EXTRACTION = "ERROR_EXTRACTION"
STATUS_ERROR_QUEUE = "ERROR_QUEUE"
STATUS_INDEXED = "INDEXED"


class DocumentMetadata(Base):
    __tablename__ = "documents"

    id = Column(Integer, primary_key=True, index=True)
    filename = Column(String, index=True)
    upload_date = Column(DateTime(timezone=True), server_default=func.now())
    status = Column(String)
    doc_type = Column(String)

    def to_dict(self) -> dict:
        return {"id": self.id, "filename": self.filename,
                "upload_date": self.upload_date.isoformat() if self.upload_date else None,
                "status": self.status, "doc_type": self.doc_type}


def database_url() -> str:
    if os.getenv("DOCQA_DB", "").lower() == "postgres":
        host, port = os.getenv("DB_HOST", "localhost"), os.getenv("DB_PORT", "5433")
        return f"postgresql://admin:adminpassword@{host}:{port}/ingestion_db"
    return os.getenv("DATABASE_URL", "sqlite:///docqa_documents.db")


class DocsDB:
    def __init__(self, url: str | None = None):
        url = url or database_url()
        kw = {}
        if url.startswith("sqlite"):
            kw["connect_args"] = {"check_same_thread": False}
            if url in ("sqlite://", "sqlite:///:memory:"):
                kw["poolclass"] = StaticPool
        self.engine = create_engine(url, **kw)
        Base.metadata.create_all(bind=self.engine)
        self.Session = sessionmaker(autocommit=False, autoflush=False, bind=self.engine,
                                    expire_on_commit=False)
        self._lock = threading.Lock()

    def create(self, filename: str, doc_type: str, status: str = STATUS_PENDING) -> int:
        with self.Session() as s:
            d = DocumentMetadata(filename=filename, status=status, doc_type=doc_type)
            s.add(d)
            s.commit()
            s.refresh(d)
            return d.id

    def set_status(self, doc_id: int, status: str) -> None:
        with self.Session() as s:
            d = s.get(DocumentMetadata, doc_id)
            if d is not None:
                d.status = status
                s.commit()

    def get(self, doc_id: int) -> dict | None:
        with self.Session() as s:
            d = s.get(DocumentMetadata, doc_id)
            return d.to_dict() if d else None

    def list(self) -> list[dict]:
        with self.Session() as s:
            return [d.to_dict() for d in s.query(DocumentMetadata).order_by(DocumentMetadata.id).all()]
