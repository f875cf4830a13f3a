"""Corpus assembly + batched index build (the semantic-indexer bootstrap path).

Reference behaviour (semantic-indexer/indexer.py:97-137): KB CSV sentences first, then
each de-identified patient document cut into fixed 500-character chunks
(``text[i:i+500]``, no overlap) labelled ``"Dossier Patient {doc_id}"`` /
``"patient_file"``; one ``model.encode([chunk])`` + ``index.add`` per chunk.
Here the chunks are embedded in large packed batches (one varlen encoder forward per
batch) and appended to the HBM-resident index in one device copy per batch.
"""
from __future__ import annotations

import torch

from ..text.chunking import chunk_chars
from ..text.kb import kb_records_from_dir, synthetic_kb_records
from ..text.synthetic import synthetic_notes


def note_records(notes: list[dict], chunk_size: int = 500) -> list[dict]:
    recs = []
    for n in notes:
        for c in chunk_chars(n["text"], chunk_size):
            recs.append({"doc_id": str(n["doc_id"]), "text_content": c,
                         "source": f"Dossier Patient {n['doc_id']}", "type": "patient_file",
                         "patient_id": n.get("patient_id")})
    return recs


def build_corpus(n_notes: int = 1000, kb_dir=None, seed: int = 0, chunk_size: int = 500) -> list[dict]:
    kb = kb_records_from_dir(kb_dir) if kb_dir else []
    if not kb:
        kb = synthetic_kb_records(seed)
    return kb + note_records(synthetic_notes(n_notes, seed), chunk_size)


@torch.inference_mode()
def embed_records(encoder, tokenizer, records: list[dict], batch: int = 512) -> torch.Tensor:
    outs = []
    for i in range(0, len(records), batch):
        toks = tokenizer.encode_batch([r["text_content"] for r in records[i:i + batch]])
        outs.append(encoder.encode(toks))
    if not outs:
        return torch.empty(0, encoder.cfg.hidden)
    return torch.cat(outs, 0)
