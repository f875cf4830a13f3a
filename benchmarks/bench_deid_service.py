"""De-identification SERVICE throughput with the NER model in the loop (VERDICT r3 item 3:
"a GPU serving run of ingest -> deid reports docs/s within 2x of bench_deid").

The deployed path, not the engine call: raw messages (the doc-ingestor's payload schema)
are published on the raw queue of the in-process broker, the DeidWorker
(services/deid_worker.py) drains up to ``--batch-docs`` of them per packed NER forward and
publishes the clean messages; docs/s is measured from the first publish to the last clean
message.  In the same process the engine-only number (DeidEngine.process_batch over the
same notes, the bench_deid.py e2e figure) is measured as the yardstick, and the JSON line
reports the ratio.  Reference: deid-service/anonymizer.py:29,41-45,97 (spaCy NER inside
Presidio, one message per callback).  Random-init clinical-BERT weights (offline).
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1024)
    ap.add_argument("--batch-docs", type=int, default=64)
    ap.add_argument("--model", default="clinical-bert")
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()

    from docqa_amd import ops
    from docqa_amd.bus.broker import InProcBroker
    from docqa_amd.config import Settings
    from docqa_amd.deid.engine import NER_LABELS, DeidEngine
    from docqa_amd.models.bert import BertConfig, BertTokenClassifier
    from docqa_amd.services.deid_worker import DeidWorker
    from docqa_amd.text.synthetic import synthetic_notes
    from docqa_amd.text.tokenizer import WordPieceTokenizer

    if a.device == "cuda":
        assert ops.load_native()
    sync = torch.cuda.synchronize if a.device == "cuda" else (lambda: None)
    cfg = BertConfig.preset(a.model)
    model = BertTokenClassifier(cfg, NER_LABELS, device=a.device)
    tok = WordPieceTokenizer(max_len=256)
    notes = synthetic_notes(a.docs, seed=9)
    texts = [n["text"] for n in notes]

    # yardstick: the engine alone (bench_deid.py's e2e figure), warm
    eng = DeidEngine(model, tok, use_model=True)
    eng.process_batch(texts[:8])
    sync()
    t = time.perf_counter()
    eng.process_batch(texts)
    sync()
    engine_dps = a.docs / (time.perf_counter() - t)

    st = Settings()
    st.deid_batch_docs = a.batch_docs
    broker = InProcBroker()
    w = DeidWorker(eng, st, broker)
    # warm the worker's path once (first forwards at these packed shapes)
    for i in range(a.batch_docs):
        broker.publish(st.raw_queue, json.dumps({"doc_id": -1 - i, "text": texts[i % a.docs],
                                                 "metadata": {"filename": "warm.txt"}}).encode())
    w.start()
    try:
        got = 0
        t_end = time.time() + 600
        while got < a.batch_docs and time.time() < t_end:
            if broker._get(st.clean_queue, timeout=0.05) is not None:
                got += 1
        b0, p0 = w.batches, w.processed
        t0 = time.perf_counter()
        for n in notes:
            broker.publish(st.raw_queue, json.dumps({"doc_id": n["doc_id"] if "doc_id" in n else 0,
                                                     "text": n["text"],
                                                     "metadata": {"filename": n["filename"]}}).encode())
        got, masked = 0, 0
        while got < a.docs and time.time() < t_end:
            m = broker._get(st.clean_queue, timeout=0.05)
            if m is not None:
                got += 1
                masked += json.loads(m[1])["original_text_masked"].count("<")
        svc_s = time.perf_counter() - t0
    finally:
        w.stop()
    assert got == a.docs, f"only {got} of {a.docs} clean messages"
    svc_dps = a.docs / svc_s
    print(json.dumps({"metric": "deid_service_docs_per_sec", "value": round(svc_dps, 1), "unit": "docs/s",
                      "engine_docs_per_s": round(engine_dps, 1),
                      "service_over_engine": round(svc_dps / engine_dps, 3),
                      "docs": a.docs, "batch_docs": a.batch_docs, "forwards": w.batches - b0,
                      "processed": w.processed - p0, "entities_masked": masked,
                      "model": f"{a.model} ({cfg.layers}x{cfg.hidden}, random init)", "device": a.device}),
          flush=True)


if __name__ == "__main__":
    main()
