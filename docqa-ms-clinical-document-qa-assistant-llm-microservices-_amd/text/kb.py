"""Knowledge-base CSV -> indexable sentences.

Reference behaviour (semantic-indexer/indexer.py:50-94): every ``*.csv`` under
``default_data`` becomes one sentence per row, one vector per sentence:
  * files whose name contains "matrice"/"ranking": a syndrome -> plant -> score sentence;
  * files whose name contains "base"/"connaissance": a clinical-detail sentence.
The reference reads a non-existent ``nom_formule`` column (so its formula is always
empty); we read ``nom_link`` -- the formula's actual column -- and fall
back to ``nom_formule`` when present.  Metadata rows keep the reference's keys
(doc_id/text_content/source/type), with ``doc_id`` the source file stem instead of the
constant ``"KB_MTC"`` (SURVEY.md §7.4 defect list).
"""
from __future__ import annotations

import csv
from pathlib import Path


def matrix_row_text(row: dict) -> str:
    return (f"ANALYSE SCORE MTC : Syndrome '{row.get('nom_syndrome', '')}'. "
            f"Plante recommandée : {row.get('nom_latin', '')} ({row.get('nom_chinois', '')}). "
            f"Score de pertinence : {row.get('score_role', '0')}.")


def base_row_text(row: dict) -> str:
    formula = row.get("nom_formule") or row.get("nom_link", "")
    return (f"DÉTAIL CLINIQUE : Syndrome '{row.get('nom_syndrome', '')}'. "
            f"Formule '{formula}'. Plante : {row.get('nom_latin', '')}. "
            f"Rôle : {row.get('role_formule', 'Inconnu') or 'Inconnu'} (Score {row.get('score_role', '')}). "
            f"Description : {row.get('description', '')}")


def row_text(filename: str, row: dict) -> str | None:
    name = filename.lower()
    if "matrice" in name or "ranking" in name:
        return matrix_row_text(row)
    if "base" in name or "connaissance" in name:
        return base_row_text(row)
    return None


def kb_records_from_rows(filename: str, rows: list[dict]) -> list[dict]:
    out = []
    for r in rows:
        t = row_text(filename, r)
        if t and t.strip():
            out.append({"doc_id": Path(filename).stem, "text_content": t, "source": filename,
                        "type": "knowledge_base"})
    return out


def kb_records_from_dir(data_dir) -> list[dict]:
    """All KB sentences from the CSVs of a directory (sorted for determinism)."""
    recs = []
    d = Path(data_dir)
    if not d.exists():
        return recs
    for p in sorted(d.glob("*.csv")):
        with open(p, encoding="utf-8") as f:
            recs.extend(kb_records_from_rows(p.name, list(csv.DictReader(f))))
    return recs


def synthetic_kb_records(seed: int = 0) -> list[dict]:
    from .synthetic import synthetic_kb

    m, b = synthetic_kb(seed=seed)
    return (kb_records_from_rows("base_connaissance_tcm.csv", b)
            + kb_records_from_rows("matrice_plante_syndrome.csv", m))
