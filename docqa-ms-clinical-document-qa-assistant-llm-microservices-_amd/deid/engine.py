"""De-identification engine: analyze -> resolve -> replace with ``<ENTITY_TYPE>``.

Reference behaviour (deid-service/anonymizer.py:37-48): empty/None -> ``""``; otherwise
Presidio analyze over six entity types followed by the default ``replace`` operator, so
every detected span becomes ``<ENTITY_TYPE>`` (confirmed by the shipped metadata rows
647-648 containing ``<NRP>`` and ``<PERSON>``).

The learned recognizer is the BERT token classifier on the MI355X (packed varlen batch of
documents, native encoder kernels, GPU argmax) whose BIO labels are decoded back to
character spans through the WordPiece offsets.  Pattern and context recognizers run on
the CPU.  Documents longer than the encoder window are split into overlapping windows.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass

from ..utils import tracing
from .recognizers import ENTITIES, Span, context_spans, pattern_spans, resolve_overlaps

NER_LABELS = ["O", "B-PER", "I-PER", "B-LOC", "I-LOC", "B-NRP", "I-NRP", "B-DATE", "I-DATE"]

# The learned recognizer of the default deployment: a 2-layer BERT token classifier trained
# from scratch on synthetic clinical notes with known PII spans (scripts/train_deid_ner.py;
# held-out names / places / nationalities in ``eval.json``).  DEID_NER=auto runs it when no
# NER_CHECKPOINT is given; a real checkpoint (NER_CHECKPOINT) replaces it.
SHIPPED_NER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", "ner-synthetic")


def shipped_ner() -> str | None:
    """Path of the shipped NER checkpoint, or None if it is missing."""
    ok = os.path.exists(os.path.join(SHIPPED_NER, "config.json")) and \
        os.path.exists(os.path.join(SHIPPED_NER, "model.safetensors"))
    return SHIPPED_NER if ok else None

# Checkpoint label type -> Presidio entity (the six entities of
# deid-service/anonymizer.py:43 plus the usual extra NER types).  Real token-classifier
# checkpoints bring their own id2label (models/checkpoint.py:load_bert_token_classifier),
# so both the CoNLL short forms (PER/LOC) and the Presidio / OntoNotes / i2b2 long forms
# are accepted.  Types mapped to None, and types missing from the table, are treated as
# "O" (skipped) rather than raising.  Extend or override with DOCQA_NER_LABEL_MAP='{"TYPE":
# "ENTITY", ...}' or the ``label_map`` argument of :class:`DeidEngine`.
DEFAULT_LABEL_ENTITY: dict[str, str | None] = {
    "PER": "PERSON", "PERSON": "PERSON", "NAME": "PERSON", "PATIENT": "PERSON",
    "DOCTOR": "PERSON", "STAFF": "PERSON", "USERNAME": "PERSON",
    "LOC": "LOCATION", "LOCATION": "LOCATION", "GPE": "LOCATION", "CITY": "LOCATION",
    "STATE": "LOCATION", "COUNTRY": "LOCATION", "STREET": "LOCATION", "ZIP": "LOCATION",
    "FAC": "LOCATION", "HOSPITAL": "LOCATION", "ADDRESS": "LOCATION",
    "NRP": "NRP", "NORP": "NRP",
    "DATE": "DATE_TIME", "DATE_TIME": "DATE_TIME", "TIME": "DATE_TIME", "AGE": None,
    "PHONE": "PHONE_NUMBER", "PHONE_NUMBER": "PHONE_NUMBER", "FAX": "PHONE_NUMBER",
    "EMAIL": "EMAIL_ADDRESS", "EMAIL_ADDRESS": "EMAIL_ADDRESS",
    "ORG": "ORGANIZATION", "ORGANIZATION": "ORGANIZATION",
    "MISC": None,
}


def label_entity_map(overrides: dict | None = None) -> dict[str, str | None]:
    """The default table, updated from ``DOCQA_NER_LABEL_MAP`` (JSON) and ``overrides``."""
    table = dict(DEFAULT_LABEL_ENTITY)
    env = os.environ.get("DOCQA_NER_LABEL_MAP")
    if env:
        table.update({str(k).upper(): v for k, v in json.loads(env).items()})
    if overrides:
        table.update({str(k).upper(): v for k, v in overrides.items()})
    return table


def _split_label(lab: str) -> tuple[str, str]:
    """'B-PER' -> ('B', 'PER'); BIOES 'S-'/'E-'/'L-'/'U-' prefixes map onto B/I;
    an un-prefixed type (IO scheme) continues the open span."""
    if len(lab) > 2 and lab[1] in "-_" and lab[0] in "BIESLU":
        tag, typ = lab[0], lab[2:]
        return ("B" if tag in "BSU" else "I"), typ
    return "I", lab


def bio_to_spans(labels: list[str], offsets: list[tuple[int, int]], score: float = 0.85,
                 label_map: dict[str, str | None] | None = None) -> list[Span]:
    """BIO tag sequence + token char offsets -> entity spans (I- without B- opens a span).
    Types the label map does not name (or maps to None) close any open span and are
    skipped, like "O"."""
    table = DEFAULT_LABEL_ENTITY if label_map is None else label_map
    spans: list[Span] = []
    cur_ent, cur_type, cur_start, cur_end = None, None, 0, 0

    def close():
        if cur_ent:
            spans.append(Span(cur_start, cur_end, cur_ent, score))

    for lab, (s, e) in zip(labels, offsets):
        if s == e:  # special token
            continue
        ent = None
        if lab != "O":
            tag, typ = _split_label(lab)
            ent = table.get(typ.upper())
        if ent is None:
            close()
            cur_ent = cur_type = None
            continue
        if tag == "B" or typ != cur_type:
            close()
            cur_ent, cur_type, cur_start, cur_end = ent, typ, s, e
        else:
            cur_end = e
    close()
    return spans


def word_labels(labels: list[str], word_ids: list) -> list[str]:
    """WordPiece -> word-level BIO: every piece of a word takes its first piece's entity
    type (I- after the first piece), so a label cannot start or stop inside a word (the
    classifier is trained on whole-word spans; a stray piece label inside "Grenoble" or
    "domicilié" would otherwise cut a span there)."""
    out = list(labels)
    prev_w, first = None, "O"
    for i, w in enumerate(word_ids[:len(labels)]):    # a model with fewer positions labels a prefix
        if w is not None and w == prev_w:
            out[i] = "O" if first == "O" else "I-" + first.split("-", 1)[-1]
        else:
            first = labels[i]
        prev_w = w
    return out


def merge_adjacent(spans: list[Span], text: str) -> list[Span]:
    """Join consecutive model spans of one entity type separated by whitespace only (a
    first name and a surname the classifier opened as two B- spans are one PERSON)."""
    out: list[Span] = []
    for sp in sorted(spans, key=lambda x: x.start):
        if out and out[-1].entity_type == sp.entity_type and sp.start >= out[-1].end \
                and text[out[-1].end:sp.start].isspace() and sp.start - out[-1].end <= 2:
            out[-1] = Span(out[-1].start, sp.end, sp.entity_type, max(out[-1].score, sp.score))
        else:
            out.append(sp)
    return out


@dataclass
class AnalyzerResult:
    entity_type: str
    start: int
    end: int
    score: float


class DeidEngine:
    def __init__(self, ner_model=None, tokenizer=None, use_model: bool = False,
                 window: int = 256, stride: int = 192, label_map: dict | None = None):
        self.ner = ner_model
        self.label_map = label_entity_map(label_map)
        self.tok = tokenizer
        self.use_model = use_model and ner_model is not None and tokenizer is not None
        self.window = window
        self.stride = stride

    # ------------------------------------------------------------------ analyze
    def _model_spans_batch(self, texts: list[str]) -> list[list[Span]]:
        """Token-classify every window of every text in ONE packed GPU forward."""
        encs = [self.tok.tok.encode(t, add_special_tokens=False) for t in texts]
        windows, owners = [], []
        for di, e in enumerate(encs):
            n = len(e.ids)
            w = self.window - 2
            starts = list(range(0, max(1, n - w + self.stride), self.stride)) or [0]
            for s0 in starts:
                windows.append((e.ids[s0:s0 + w], e.offsets[s0:s0 + w], e.word_ids[s0:s0 + w]))
                owners.append(di)
                if s0 + w >= n:
                    break
        cls = self.tok.tok.token_to_id("[CLS]") or 2
        sep = self.tok.tok.token_to_id("[SEP]") or 3
        toks = [[cls] + ids + [sep] for ids, _, _ in windows]
        preds = self.ner.predict(toks) if toks else []
        out: list[list[Span]] = [[] for _ in texts]
        for (ids, offs, wids), owner, p in zip(windows, owners, preds):
            labels = [self.ner.labels[i] if i < len(self.ner.labels) else "O" for i in p[1:-1]]
            labels = word_labels(labels, list(wids))
            out[owner] += bio_to_spans(labels, list(offs), label_map=self.label_map)
        return [merge_adjacent(sp, t) for sp, t in zip(out, texts)]

    def analyze_batch(self, texts: list[str], entities=None) -> list[list[AnalyzerResult]]:
        ents = list(entities or ENTITIES)
        model = self._model_spans_batch(texts) if self.use_model else [[] for _ in texts]
        res = []
        for t, ms in zip(texts, model):
            spans = pattern_spans(t, ents) + context_spans(t, ents) + [s for s in ms if s.entity_type in ents]
            res.append([AnalyzerResult(s.entity_type, s.start, s.end, s.score) for s in resolve_overlaps(spans)])
        return res

    def analyze(self, text: str, entities=None, language: str = "en") -> list[AnalyzerResult]:
        return self.analyze_batch([text], entities)[0]

    # ------------------------------------------------------------------ anonymize
    @staticmethod
    def anonymize(text: str, results: list[AnalyzerResult]) -> str:
        out, last = [], 0
        for r in sorted(results, key=lambda r: r.start):
            if r.start < last:
                continue
            out.append(text[last:r.start])
            out.append(f"<{r.entity_type}>")
            last = r.end
        out.append(text[last:])
        return "".join(out)

    def process_batch(self, texts: list[str], entities=None) -> list[str]:
        with tracing.span("deid.analyze", docs=len(texts), model=self.use_model):
            res = self.analyze_batch([t or "" for t in texts], entities)
        return ["" if not t else self.anonymize(t, r) for t, r in zip(texts, res)]

    def process_text_anonymization(self, text, entities=None) -> str:
        """Reference-compatible entry point (deid-service/anonymizer.py:37-48)."""
        if not text:
            return ""
        return self.process_batch([text], entities)[0]
