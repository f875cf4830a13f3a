"""patient-snippets time window (synthese-comparative/core/retrieval_client.py:81-89 sends
from_date / to_date): the note date is taken from the raw text at ingest (text/dates.py),
carried in the queue metadata, stored per chunk and filtered on by the indexer."""
import torch

from docqa_amd.text.dates import first_date, in_window, parse_date


def test_parse_and_first_date():
    assert parse_date("2021-03-12") == "2021-03-12"
    assert parse_date("12/03/2021") == "2021-03-12"
    assert parse_date("5.7.2019") == "2019-07-05"
    assert parse_date("1er mars 2020") == "2020-03-01"
    assert parse_date("2024-01-02T10:00:00") == "2024-01-02"
    assert parse_date("hier") is None and parse_date(None) is None
    assert parse_date("31/13/2020") is None
    text = "Compte-rendu de consultation du 14/02/2022.\\nPatient né le 03/04/1961. Contrôle le 2022-05-01."
    assert first_date(text) == "2022-02-14"
    assert first_date("pas de date") is None
    assert in_window("2022-02-14", "2022-01-01", None) and not in_window("2021-12-31", "2022-01-01", "2022-12-31")
    assert in_window(None, None, None) and not in_window(None, "2022-01-01", None)


def test_patient_snippets_date_window(tmp_path):
    from docqa_amd.config import Settings
    from docqa_amd.models.bert import BertConfig, BertEncoder
    from docqa_amd.services.indexer import SemanticIndexer
    from docqa_amd.text.tokenizer import WordPieceTokenizer

    st = Settings()
    st.index_dir = str(tmp_path)
    enc = BertEncoder(BertConfig.preset("tiny-bert"), device="cpu")
    idx = SemanticIndexer(enc, WordPieceTokenizer(), st, device="cpu").startup(build_if_missing=False)
    notes = [("2021-03-12", "anticoagulant warfarine"), ("2022-06-01", "insomnie"), ("2023-11-20", "fatigue")]
    for i, (d, t) in enumerate(notes):
        idx.index_document(i + 1, f"Note {i}: {t}", {"patient_id": "P7", "note_date": d})
    idx.index_document(9, "autre patient", {"patient_id": "P8", "note_date": "2022-01-01"})
    allp = idx.patient_snippets("P7")
    assert [s["doc_id"] for s in allp] == ["1", "2", "3"]
    assert [s["doc_id"] for s in idx.patient_snippets("P7", "2022-01-01", None)] == ["2", "3"]
    assert [s["doc_id"] for s in idx.patient_snippets("P7", None, "01/07/2022")] == ["1", "2"]
    assert [s["doc_id"] for s in idx.patient_snippets("P7", "2022-01-01", "2022-12-31")] == ["2"]
    with torch.inference_mode():
        got = idx.patient_snippets("P7", "2021-01-01", "2023-12-31", focus="insomnie")
    assert sorted(s["doc_id"] for s in got) == ["1", "2", "3"]
