"""PII recognizers for the deid-service.

Pattern recognizers (CPU, regex + checksum-free validation) cover EMAIL_ADDRESS,
PHONE_NUMBER and DATE_TIME; context/gazetteer recognizers cover PERSON, LOCATION and
NRP (nationality / religious / political group).  The learned path -- the BERT token
classifier on the MI355X (``models/bert.py:BertTokenClassifier``) -- contributes spans
for PERSON/LOCATION/NRP/DATE_TIME when trained weights are loaded.

Reference parity: Presidio ``AnalyzerEngine.analyze(text, entities=[PERSON,
PHONE_NUMBER, EMAIL_ADDRESS, DATE_TIME, NRP, LOCATION], language=NLP_LANG)``
(deid-service/anonymizer.py:41-45), which combines spaCy NER with regex recognizers.
Scores mimic Presidio's convention (pattern 0.5-1.0, NER 0.85).
"""
from __future__ import annotations

import re
from dataclasses import dataclass

ENTITIES = ["PERSON", "PHONE_NUMBER", "EMAIL_ADDRESS", "DATE_TIME", "NRP", "LOCATION"]


@dataclass(frozen=True)
class Span:
    start: int
    end: int
    entity_type: str
    score: float

    def __len__(self) -> int:
        return self.end - self.start


EMAIL_RE = re.compile(r"\b[A-Za-z0-9._%+-]+@[A-Za-z0-9.-]+\.[A-Za-z]{2,}\b")
PHONE_RE = re.compile(
    r"(?<![\w/])(?:\+\d{1,3}[\s.-]?)?(?:\(?0?\d{1,3}\)?[\s.-]?)?\d{2}(?:[\s.-]?\d{2}){3,4}(?![\w/])")
DATE_RES = [
    re.compile(r"\b\d{1,2}[/.-]\d{1,2}[/.-]\d{2,4}\b"),
    re.compile(r"\b\d{4}-\d{2}-\d{2}(?:[T ]\d{2}:\d{2}(?::\d{2})?)?\b"),
    re.compile(r"\b\d{1,2}(?:er)?\s+(?:janvier|février|fevrier|mars|avril|mai|juin|juillet|août|aout|"
               r"septembre|octobre|novembre|décembre|decembre|january|february|march|april|may|june|"
               r"july|august|september|october|november|december)\s+\d{4}\b", re.I),
    re.compile(r"\b(?:[01]?\d|2[0-3])[h:][0-5]\d\b"),
]

NATIONALITIES = {
    "française", "français", "marocaine", "marocain", "algérienne", "algérien", "belge", "suisse",
    "canadienne", "canadien", "tunisienne", "tunisien", "sénégalaise", "sénégalais", "italienne",
    "italien", "espagnole", "espagnol", "allemande", "allemand", "américaine", "américain",
    "french", "moroccan", "algerian", "belgian", "swiss", "canadian", "american", "german",
    "musulman", "musulmane", "chrétien", "chrétienne", "juif", "juive", "catholique", "protestant",
}
CITIES = {
    "paris", "lyon", "marseille", "toulouse", "casablanca", "rabat", "lille", "nantes", "bordeaux",
    "montréal", "montreal", "genève", "geneve", "bruxelles", "strasbourg", "nice", "fès", "fes",
    "tanger", "marrakech", "alger", "tunis", "dakar", "london", "new york", "rennes", "grenoble",
}
_TITLE = r"(?:Dr\.?|Docteur|Pr\.?|Professeur|M\.|Mr\.?|Mme\.?|Mlle\.?|Madame|Monsieur|Mrs\.?|Ms\.?)"
_NAME = r"[A-ZÉÈÀÂÎÔÛÇ][a-zéèêëàâîïôöûüç'-]+"
PERSON_TITLE_RE = re.compile(rf"{_TITLE}\s+((?:{_NAME})(?:\s+{_NAME}){{0,2}})")
PERSON_FIELD_RE = re.compile(rf"(?:Patient|Patiente|Nom|Name|Médecin|Medecin)\s*:\s*((?:{_NAME})(?:\s+{_NAME}){{0,2}})")
LOCATION_CTX_RE = re.compile(rf"\b(?:à|a|de|in|at)\s+({_NAME}(?:[\s-]{_NAME})?)")


def pattern_spans(text: str, entities=None) -> list[Span]:
    want = set(entities or ENTITIES)
    out: list[Span] = []
    if "EMAIL_ADDRESS" in want:
        out += [Span(m.start(), m.end(), "EMAIL_ADDRESS", 1.0) for m in EMAIL_RE.finditer(text)]
    if "DATE_TIME" in want:
        for rx in DATE_RES:
            out += [Span(m.start(), m.end(), "DATE_TIME", 0.85) for m in rx.finditer(text)]
    if "PHONE_NUMBER" in want:
        for m in PHONE_RE.finditer(text):
            digits = re.sub(r"\D", "", m.group())
            if 9 <= len(digits) <= 15:
                out.append(Span(m.start(), m.end(), "PHONE_NUMBER", 0.75))
    return out


def context_spans(text: str, entities=None) -> list[Span]:
    want = set(entities or ENTITIES)
    out: list[Span] = []
    if "PERSON" in want:
        for rx in (PERSON_TITLE_RE, PERSON_FIELD_RE):
            out += [Span(m.start(1), m.end(1), "PERSON", 0.85) for m in rx.finditer(text)]
    if "NRP" in want:
        for m in re.finditer(r"[\wéèêàâîôûç]+", text):
            if m.group().lower() in NATIONALITIES:
                out.append(Span(m.start(), m.end(), "NRP", 0.85))
    if "LOCATION" in want:
        low = text.lower()
        for city in CITIES:
            for m in re.finditer(rf"\b{re.escape(city)}\b", low):
                out.append(Span(m.start(), m.end(), "LOCATION", 0.85))
        for m in LOCATION_CTX_RE.finditer(text):
            if m.group(1).lower() in CITIES:
                out.append(Span(m.start(1), m.end(1), "LOCATION", 0.85))
    return out


def resolve_overlaps(spans: list[Span]) -> list[Span]:
    """Presidio-style conflict resolution: among overlapping spans keep the highest
    score, then the longest, then the earliest; identical duplicates collapse."""
    ordered = sorted(set(spans), key=lambda s: (-s.score, -len(s), s.start))
    kept: list[Span] = []
    for s in ordered:
        if all(s.end <= k.start or s.start >= k.end for k in kept):
            kept.append(s)
    return sorted(kept, key=lambda s: s.start)
