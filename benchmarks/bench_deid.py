"""BASELINE.json config 3: deid-service clinical-BERT NER token classification, batched
forward on one MI355X.

Input: synthetic French clinical notes (with names, dates, phones, e-mails, cities) split
into 256-token windows, packed varlen (no padding) -- the same path
``DeidEngine._model_spans_batch`` uses.  Measured: NER forward throughput (windows/s,
tokens/s) at several batch sizes, plus end-to-end de-identification docs/s (tokenise +
NER on the GPU + pattern/context recognizers + span resolution + replacement).
Random-init weights (no clinical checkpoint is reachable offline).  One JSON line.
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
    ap.add_argument("--docs", type=int, default=512)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--model", default="clinical-bert")
    a = ap.parse_args()
    from docqa_amd import ops
    from docqa_amd.deid.engine import NER_LABELS, DeidEngine
    from docqa_amd.models.bert import BertConfig, BertTokenClassifier, pack
    from docqa_amd.text.synthetic import synthetic_notes
    from docqa_amd.text.tokenizer import WordPieceTokenizer

    assert ops.load_native()
    cfg = BertConfig.preset(a.model)
    model = BertTokenClassifier(cfg, NER_LABELS, device="cuda")
    tok = WordPieceTokenizer(max_len=256)
    notes = [n["text"] for n in synthetic_notes(a.docs, seed=9)]
    toks = tok.encode_batch(notes)
    ntok = sum(len(t) for t in toks)
    res = {}
    for bs in (8, 64, 256):
        batch = (toks * ((bs // len(toks)) + 1))[:bs]
        ids, cu, ml = pack(batch, 256, "cuda")
        model.predict_packed(ids, cu, ml)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            model.predict_packed(ids, cu, ml)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.iters
        nt = int(cu[-1])
        res[f"batch{bs}"] = {"ms": round(dt * 1e3, 3), "seq_per_s": round(bs / dt, 1),
                             "tokens_per_s": round(nt / dt, 1)}
    eng = DeidEngine(model, tok, use_model=True)
    eng.process_batch(notes[:8])
    torch.cuda.synchronize()
    t = time.perf_counter()
    outs = eng.process_batch(notes)
    torch.cuda.synchronize()
    e2e = time.perf_counter() - t
    masked = sum(o.count("<") for o in outs)
    print(json.dumps({"metric": "deid_ner_throughput", "model": f"{a.model} ({cfg.layers}x{cfg.hidden})",
                      "ner_forward": res, "e2e_docs_per_s": round(a.docs / e2e, 1),
                      "e2e_tokens_per_s": round(ntok / e2e, 1), "entities_masked": masked}), flush=True)


if __name__ == "__main__":
    main()
