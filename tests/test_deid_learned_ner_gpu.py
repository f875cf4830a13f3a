"""The shipped learned de-identification NER (deid/assets/ner-synthetic) on the GPU: the
encoder kernels + fused token-classification head + argmax in bf16 find the same entities
as the fp32 CPU forward on notes none of whose names, places or nationalities it saw in
training (tests/test_deid_learned_ner_cpu.py holds the CPU side)."""
import pytest
import torch

from docqa_amd import ops
from docqa_amd.deid.engine import NER_LABELS, SHIPPED_NER, DeidEngine, shipped_ner
from docqa_amd.models import checkpoint as ck
from docqa_amd.text.tokenizer import WordPieceTokenizer

pytestmark = pytest.mark.gpu

TEXTS = [
    "Compte-rendu de consultation du 14/02/2023. Patient : Gontran Vasseur, né le 3 mars 1961 à Besançon, "
    "nationalité luxembourgeoise. Suivi par le Dr Ophélie Carpentier à Colmar.",
    "Patiente : Prune Lavergne, née le 12/05/1958 à Quimper. Motif : fatigue et insomnie depuis 6 semaines.",
    "Referred by Dr. Anselme Broussard at Perpignan. Visit on 2021-11-03. Famille portugaise, vit à Annecy.",
]


def _spans(engine, text):
    return {(text[s.start:s.end], s.entity_type) for s in engine._model_spans_batch([text])[0]}


def test_shipped_ner_gpu_matches_cpu():
    assert ops.load_native()
    assert shipped_ner() is not None
    tok = WordPieceTokenizer()
    gpu = DeidEngine(ck.load_bert_token_classifier(SHIPPED_NER, NER_LABELS, device="cuda"), tok, use_model=True)
    cpu = DeidEngine(ck.load_bert_token_classifier(SHIPPED_NER, NER_LABELS, device="cpu"), tok, use_model=True)
    assert gpu.ner.dtype == torch.bfloat16
    for t in TEXTS:
        g, c = _spans(gpu, t), _spans(cpu, t)
        assert len(g & c) >= 0.9 * max(len(c), 1), (t, g, c)
    got = _spans(gpu, TEXTS[0])
    for want in [("Gontran Vasseur", "PERSON"), ("Besançon", "LOCATION"), ("3 mars 1961", "DATE_TIME")]:
        assert want in got, (want, got)
