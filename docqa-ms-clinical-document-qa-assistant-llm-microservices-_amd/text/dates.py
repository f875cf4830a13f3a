"""Clinical note dates: the ``patient-snippets`` time window filter of the semantic-indexer
(synthese-comparative/core/retrieval_client.py:81-89 sends ``from_date`` / ``to_date``).

De-identification replaces the dates INSIDE a note with ``<DATE_TIME>``, so the note's
date is taken at ingest, from the raw text (the first clinical date it states, e.g.
"Compte-rendu de consultation du 12/03/2021"), and travels in the queue message's
metadata as ``note_date`` (ISO ``YYYY-MM-DD``) -- the reference's consumers pass metadata
through unchanged.
"""
from __future__ import annotations

import re

_DMY = re.compile(r"(?<!\d)(\d{1,2})[/.\-](\d{1,2})[/.\-](\d{4})(?!\d)")
_YMD = re.compile(r"(?<!\d)(\d{4})-(\d{1,2})-(\d{1,2})(?!\d)")
_MONTHS = {"janvier": 1, "février": 2, "fevrier": 2, "mars": 3, "avril": 4, "mai": 5, "juin": 6, "juillet": 7,
           "août": 8, "aout": 8, "septembre": 9, "octobre": 10, "novembre": 11, "décembre": 12, "decembre": 12}
_FR = re.compile(r"\b(\d{1,2})(?:er)?\s+(" + "|".join(_MONTHS) + r")\s+(\d{4})\b", re.IGNORECASE)


def _iso(y: int, m: int, d: int) -> str | None:
    if 1 <= m <= 12 and 1 <= d <= 31 and 1900 <= y <= 2100:
        return f"{y:04d}-{m:02d}-{d:02d}"
    return None


def parse_date(s: str | None) -> str | None:
    """ISO date of a query parameter / metadata value: YYYY-MM-DD[...], DD/MM/YYYY,
    DD-MM-YYYY, DD.MM.YYYY or "12 mars 2021"; None when unparseable."""
    if not s:
        return None
    s = str(s).strip()
    m = _YMD.match(s)
    if m:
        return _iso(int(m[1]), int(m[2]), int(m[3]))
    m = _DMY.match(s)
    if m:
        return _iso(int(m[3]), int(m[2]), int(m[1]))
    m = _FR.match(s)
    if m:
        return _iso(int(m[3]), _MONTHS[m[2].lower()], int(m[1]))
    return None


def first_date(text: str) -> str | None:
    """The earliest-positioned date stated in ``text`` (ISO), None if there is none."""
    best = None
    for rx, conv in ((_DMY, lambda m: _iso(int(m[3]), int(m[2]), int(m[1]))),
                     (_YMD, lambda m: _iso(int(m[1]), int(m[2]), int(m[3]))),
                     (_FR, lambda m: _iso(int(m[3]), _MONTHS[m[2].lower()], int(m[1])))):
        for m in rx.finditer(text or ""):
            iso = conv(m)
            if iso and (best is None or m.start() < best[0]):
                best = (m.start(), iso)
            break
    return best[1] if best else None


def in_window(date: str | None, lo: str | None, hi: str | None) -> bool:
    """``date`` (ISO) inside [lo, hi] (either bound optional); an undated record is outside
    any window that has a bound."""
    if lo is None and hi is None:
        return True
    if date is None:
        return False
    return (lo is None or date >= lo) and (hi is None or date <= hi)
