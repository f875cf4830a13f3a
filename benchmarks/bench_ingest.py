"""BASELINE.json config 1: doc-ingestor -> semantic-indexer, MiniLM-L6 embed + flat L2
search, 1k synthetic notes -- the plumbing benchmark (CPU by default, ``--device cuda``
for the same path on the GPU kernels).

The whole ingestion chain of the reference runs in-process with its real message flow
(SURVEY.md §3.1): ``POST /ingest/`` (multipart upload, DB row, text extraction, publish to
raw_documents_queue) -> de-identification worker (regex + gazetteer recognisers; the NER
model is off here as in config 1) -> clean_documents_queue -> semantic indexer (500-char
chunks, MiniLM-L6 architecture with random-init weights, flat L2 index) -> status
INDEXED.  Reports documents/s and chunks/s from the first upload to the last INDEXED
status, then search latency through ``POST /api/search`` and the raw index QPS.
One JSON line.
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--notes", type=int, default=1000)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--queries", type=int, default=64)
    a = ap.parse_args()

    import torch
    from fastapi.testclient import TestClient

    from docqa_amd.config import Settings
    from docqa_amd.services.multipart import FilePart, encode_multipart
    from docqa_amd.services.stack import DocQAStack, StackOptions
    from docqa_amd.store import docs_db
    from docqa_amd.text.synthetic import synthetic_notes, synthetic_questions

    if a.device == "cuda":
        from docqa_amd import ops
        assert ops.load_native()
    import tempfile
    tmp = tempfile.mkdtemp(prefix="docqa_ingest_bench_")
    st = Settings()
    st.database_url = f"sqlite:///{tmp}/docs.db"
    st.index_dir = tmp
    st.upload_dir = f"{tmp}/uploads"
    stack = DocQAStack(StackOptions(llm="tiny", embed="minilm-l6", device=a.device, use_graphs=False,
                                    max_batch=4, max_context=1024), st)
    try:
        kb_vectors = stack.indexer.index.ntotal      # knowledge base bootstrapped at startup
        notes = synthetic_notes(a.notes, seed=7)
        ing = TestClient(stack.ingest_app)
        t0 = time.perf_counter()
        ids = []
        for n in notes:
            body, ct = encode_multipart({"file": FilePart(n["filename"], "text/plain", n["text"].encode()),
                                         "doc_type": n["doc_type"]})
            r = ing.post("/ingest/", content=body, headers={"content-type": ct})
            ids.append(r.json()["doc_id"])
        t_upload = time.perf_counter() - t0
        deadline = time.time() + 1800
        want = set(ids)
        while time.time() < deadline:
            done = {d["id"] for d in stack.db.list() if d["status"] == docs_db.STATUS_INDEXED}
            if want <= done:
                break
            time.sleep(0.05)
        t_all = time.perf_counter() - t0
        chunks = stack.indexer.index.ntotal - kb_vectors
        # search through the HTTP API (one request at a time, like the reference retriever)
        idx = TestClient(stack.indexer_app)
        qs = synthetic_questions(a.queries, seed=3)
        idx.post("/api/search", json={"query": qs[0], "k": 3})
        lat = []
        for q in qs:
            t = time.perf_counter()
            r = idx.post("/api/search", json={"query": q, "k": 3})
            lat.append(time.perf_counter() - t)
            assert r.status_code == 200 and len(r.json()) == 3
        # raw index throughput on a batch of query embeddings
        qe = stack.encoder.encode(stack.enc_tok.encode_batch(qs))
        if a.device == "cuda":
            torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            stack.indexer.index.search(qe, 3)
        if a.device == "cuda":
            torch.cuda.synchronize()
        raw_qps = 10 * len(qs) / (time.perf_counter() - t)
        out = {"metric": "ingest_docs_per_sec", "config": f"config1 {a.notes} synthetic notes, MiniLM-L6 "
               f"(random init), flat L2, device={a.device}",
               "value": round(len(ids) / t_all, 2), "unit": "docs/s",
               "upload_s": round(t_upload, 2), "ingest_to_indexed_s": round(t_all, 2),
               "chunks": chunks, "chunks_per_sec": round(chunks / t_all, 1),
               "search_api_p50_ms": round(1e3 * statistics.median(lat), 2),
               "search_api_p99_ms": round(1e3 * sorted(lat)[int(0.99 * (len(lat) - 1))], 2),
               "raw_index_qps_batch": round(raw_qps, 1)}
        print(json.dumps(out), flush=True)
    finally:
        stack.close()


if __name__ == "__main__":
    main()
