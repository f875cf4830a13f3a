"""clinical-ui proxy app (services/ui.py, reference clinical-ui/app.py:1-118) and the prompt
templates (services/synthese.py, pipeline/rag.py; reference synthese-comparative/api/
routes.py:45-101 and llm-qa/main.py:72-95).  The UI's upstream calls go to an
httpx.MockTransport, so no server is started."""
import json
from pathlib import Path

import httpx
import pytest
from fastapi.testclient import TestClient

import docqa_amd.services.ui as ui


@pytest.fixture
def upstream(monkeypatch):
    """Fake doc-ingestor (port 8000) + llm-qa (port 8001); records the requests."""
    seen = []

    def handler(req: httpx.Request) -> httpx.Response:
        seen.append(req)
        host, path = req.url.port, req.url.path
        if path == "/health":
            return httpx.Response(200, json={"status": "ok"}) if host == 8000 else httpx.Response(500)
        if host == 8000 and path == "/ingest/":
            return httpx.Response(200, json={"doc_id": 7, "status": "PENDING"})
        if host == 8000 and path == "/documents/7":
            return httpx.Response(200, json={"id": 7, "status": "INDEXED"})
        if host == 8001 and path == "/ask/":
            q = json.loads(req.content)["question"]
            if q == "no-index":
                return httpx.Response(503, json={"detail": "Index non chargé."})
            return httpx.Response(200, json={"answer": f"re: {q}", "sources": ["Dossier Patient 1"]})
        return httpx.Response(404, json={"detail": "not found"})

    real = httpx.AsyncClient

    class Mocked(real):
        def __init__(self, *a, **kw):
            kw["transport"] = httpx.MockTransport(handler)
            super().__init__(*a, **kw)

    monkeypatch.setattr(ui.httpx, "AsyncClient", Mocked)
    return seen


def test_ui_page_wires_the_reference_flows():
    c = TestClient(ui.create_app())
    html = c.get("/").text
    for needle in ("/ui/health", "/ui/ingest", "/ui/ask", "/ui/documents/", "compte-rendu", "Sources"):
        assert needle in html


def test_ui_health_probes_each_service(upstream):
    c = TestClient(ui.create_app())
    assert c.get("/ui/health").json() == {"doc-ingestor": True, "llm-qa": False}


def test_ui_upload_and_readiness_poll(upstream):
    c = TestClient(ui.create_app())
    r = c.post("/ui/ingest", files={"file": ("note.txt", b"Patient: Jean", "text/plain")},
               data={"doc_type": "compte-rendu"})
    assert r.status_code == 200 and r.json()["doc_id"] == 7
    fwd = [q for q in upstream if q.url.path == "/ingest/"][0]
    assert fwd.headers["content-type"].startswith("multipart/form-data")
    assert b"compte-rendu" in fwd.content and b"Patient: Jean" in fwd.content
    assert c.get("/ui/documents/7").json()["status"] == "INDEXED"


def test_ui_ask_proxies_answer_and_errors(upstream):
    c = TestClient(ui.create_app())
    r = c.post("/ui/ask", json={"question": "dose ?"})
    assert r.json() == {"answer": "re: dose ?", "sources": ["Dossier Patient 1"]}
    r = c.post("/ui/ask", json={"question": "no-index"})
    assert r.status_code == 503 and r.json()["detail"] == "Index non chargé."


def test_synthese_templates_have_the_reference_slots():
    from docqa_amd.services.synthese import MULTI_PATIENT_TEMPLATE, SINGLE_PATIENT_TEMPLATE

    s = SINGLE_PATIENT_TEMPLATE.format(patient_alias="PATIENT_1", from_date="N/A", to_date="N/A",
                                       focus="diabète", documents="[d1]\nnote")
    assert "PATIENT_1" in s and "diabète" in s and "[d1]\nnote" in s
    for sec in ("Contexte général", "Focus clinique (diabète)", "Événements clés", "Points de vigilance"):
        assert sec in s
    m = MULTI_PATIENT_TEMPLATE.format(patients="PATIENT_1, PATIENT_2", from_date="N/A", to_date="N/A",
                                      focus="général", documents_by_patient="=== PATIENT_1 ===\n...")
    assert "PATIENT_1, PATIENT_2" in m and "=== PATIENT_1 ===" in m


def test_rag_template_puts_fixed_text_first_for_the_prefix_cache():
    """The cache-friendly template: two questions with different contexts share every
    token up to the context slot.  (The service default is the verbatim reference text.)"""
    from docqa_amd import prompts
    from docqa_amd.pipeline.rag import DEFAULT_TEMPLATE as SERVICE_DEFAULT
    from docqa_amd.text.tokenizer import ChatTokenizer

    assert SERVICE_DEFAULT is prompts.REFERENCE_QA_TEMPLATE
    DEFAULT_TEMPLATE = prompts.CACHE_FRIENDLY_QA_TEMPLATE

    assert DEFAULT_TEMPLATE.index("{context}") < DEFAULT_TEMPLATE.index("{question}")
    head = DEFAULT_TEMPLATE.split("{context}")[0]
    assert len(head) > 400                       # the shared instruction block
    tok = ChatTokenizer(model_vocab=128256)
    a = tok.chat_prompt(DEFAULT_TEMPLATE.format(context="Ginseng score 10", question="Quelle plante ?"))
    b = tok.chat_prompt(DEFAULT_TEMPLATE.format(context="Réglisse score 7", question="Posologie ?"))
    common = next(i for i, (x, y) in enumerate(zip(a, b)) if x != y)
    assert common >= len(tok.chat_prompt(head)) - 8


def test_prompt_pieces_identical_to_full_tokenisation(monkeypatch):
    """RAG prompts assembled from cached per-chunk token ids equal the token ids of the
    formatted prompt (the byte-level BPE does not merge across the paragraph breaks the
    pieces are split at)."""
    import torch

    from docqa_amd.pipeline.rag import RAGPipeline
    from docqa_amd.text.synthetic import synthetic_questions
    from docqa_amd.text.tokenizer import ChatTokenizer

    tok = ChatTokenizer(model_vocab=128256)
    meta = [{"text_content": f"Patient {i} : toux chronique, fatigue ; Ren Shen (score {i % 10}).",
             "source": f"s{i}"} for i in range(20)]

    class _Eng:
        device = torch.device("cpu")

    pipe = RAGPipeline(None, None, None, meta, _Eng(), tok)
    qs = synthetic_questions(24, seed=3)
    I = [[(7 * j + r) % 20 for r in range(3)] for j in range(len(qs))]
    monkeypatch.setenv("DOCQA_PROMPT_PIECES", "0")
    full = pipe.build_prompts(qs, I)
    monkeypatch.setenv("DOCQA_PROMPT_PIECES", "1")
    assert pipe.build_prompts(qs, I) == full
    assert tok.encode_batch_chat([qs[0]]) == [tok.chat_prompt(qs[0])]


def test_shared_context_order():
    """context_order="shared": each prompt holds the same chunks, the batch's most
    retrieved first (ties by id), so prompts with a common chunk share a token prefix;
    "relevance" keeps the retrieval order."""
    import torch

    from docqa_amd.pipeline.rag import RAGPipeline
    from docqa_amd.text.tokenizer import ChatTokenizer

    tok = ChatTokenizer(model_vocab=128256)
    meta = [{"text_content": f"Note {i} : toux, fatigue ; Ren Shen (score {i % 10}).", "source": f"s{i}"}
            for i in range(10)]

    class _Eng:
        device = torch.device("cpu")

    I = [[3, 7, 1], [9, 7, 2], [7, 5, 3]]
    rel = RAGPipeline(None, None, None, meta, _Eng(), tok, context_order="relevance")
    sh = RAGPipeline(None, None, None, meta, _Eng(), tok, context_order="shared")
    assert rel._ordered(I) == I
    assert sh._ordered(I) == [[7, 3, 1], [7, 2, 9], [7, 3, 5]]
    a, b = sh.build_prompts(["q1", "q2"], [[3, 7, 1], [9, 7, 2]])
    ra, rb = rel.build_prompts(["q1", "q2"], [[3, 7, 1], [9, 7, 2]])
    common = lambda x, y: next(i for i, (u, v) in enumerate(zip(x, y)) if u != v)   # noqa: E731
    assert common(a, b) > common(ra, rb) + 10           # chunk 7 is shared in the new order
    assert sorted(a) == sorted(ra)                      # same tokens, other order
    with pytest.raises(ValueError):
        RAGPipeline(None, None, None, meta, _Eng(), tok, context_order="random")


REF = Path("/root/reference")


def _ref_template(path: Path, marker: str) -> str:
    src = path.read_text(encoding="utf-8")
    i = src.index(marker) + len(marker)
    return src[i:src.index('"""', i)]


@pytest.mark.skipif(not (REF / "llm-qa" / "main.py").exists(), reason="reference not mounted")
def test_reference_prompts_verbatim():
    """The QA template selectable with QA_TEMPLATE=reference and the synthese templates are
    byte-identical to the reference's (llm-qa/main.py:71-93, core/prompts.py:3-45)."""
    from docqa_amd import prompts

    assert prompts.REFERENCE_QA_TEMPLATE == _ref_template(REF / "llm-qa" / "main.py", 'template = """')
    pr = REF / "synthese-comparative" / "core" / "prompts.py"
    assert prompts.SINGLE_PATIENT_TEMPLATE == _ref_template(pr, 'SINGLE_PATIENT_TEMPLATE = """')
    assert prompts.MULTI_PATIENT_TEMPLATE == _ref_template(pr, 'MULTI_PATIENT_TEMPLATE = """')
    from docqa_amd.services import synthese
    assert synthese.SINGLE_PATIENT_TEMPLATE is prompts.SINGLE_PATIENT_TEMPLATE
    assert synthese.MULTI_PATIENT_TEMPLATE is prompts.MULTI_PATIENT_TEMPLATE


def test_qa_template_selection(monkeypatch):
    import torch

    from docqa_amd import prompts
    from docqa_amd.pipeline.rag import RAGPipeline
    from docqa_amd.text.tokenizer import ChatTokenizer

    class _Eng:
        device = torch.device("cpu")

    tok = ChatTokenizer(model_vocab=128256)
    meta = [{"text_content": f"Ren Shen score {i}", "source": f"s{i}"} for i in range(4)]
    monkeypatch.setenv("QA_TEMPLATE", "reference")
    p = RAGPipeline(None, None, None, meta, _Eng(), tok)
    assert p.template is prompts.REFERENCE_QA_TEMPLATE
    # the piece-wise prompt assembly is exact for the reference order too
    I = [[0, 1, 2], [3, 2, 1]]
    qs = ["Quelle plante ?", "Posologie pour P00042 ?"]
    monkeypatch.setenv("DOCQA_PROMPT_PIECES", "0")
    full = p.build_prompts(qs, I)
    monkeypatch.setenv("DOCQA_PROMPT_PIECES", "1")
    assert p.build_prompts(qs, I) == full
    monkeypatch.setenv("QA_TEMPLATE", "cache_friendly")
    assert RAGPipeline(None, None, None, meta, _Eng(), tok).template is prompts.CACHE_FRIENDLY_QA_TEMPLATE
    with pytest.raises(ValueError):
        prompts.qa_template("nope")


def test_unique_questions_are_distinct():
    from docqa_amd.text.synthetic import synthetic_questions, synthetic_unique_questions

    qs = synthetic_unique_questions(6400, seed=123)
    assert len(set(qs)) == 6400
    assert synthetic_unique_questions(50, seed=123) == qs[:50]
    assert len(set(synthetic_questions(6400, seed=123))) < 1000   # the cache-hot grid


def test_trie_context_order_reuses_earlier_orders():
    """context_order="trie": a prompt whose chunk set has a leading order an earlier prompt
    already used (same or earlier batch) takes that order; otherwise popularity order."""
    import torch

    from docqa_amd.pipeline.rag import RAGPipeline
    from docqa_amd.text.tokenizer import ChatTokenizer

    tok = ChatTokenizer(model_vocab=128256)
    meta = [{"text_content": f"Note {i}.", "source": f"s{i}"} for i in range(10)]

    class _Eng:
        device = torch.device("cpu")

    p = RAGPipeline(None, None, None, meta, _Eng(), tok, context_order="trie")
    assert p._ordered([[3, 7, 1]]) == [[1, 3, 7]]              # no history: popularity, ids
    # batch popularity (5 and 8 twice) leads; the second prompt shares the pair (5, 8)
    assert p._ordered([[5, 8, 2], [8, 6, 5]]) == [[5, 8, 2], [5, 8, 6]]
    # a later batch: id / popularity order would be (2, 5, 8); the order an earlier prompt
    # used -- whose KV the prefix cache holds -- wins
    assert p._ordered([[2, 8, 5]]) == [[5, 8, 2]]
    assert p._ordered([[1, 9, 3]]) == [[1, 3, 9]]              # longest known prefix (1, 3)
    rel = RAGPipeline(None, None, None, meta, _Eng(), tok)     # reference template default
    assert rel.context_order == "relevance"


def test_shipped_tokenizer_vocabularies(monkeypatch, tmp_path):
    """The trained vocabularies ship with the package and are loaded in preference to a
    training run, so every machine tokenises (and retrieves, and prompts) identically."""
    import json

    from docqa_amd.text import tokenizer as T

    for name in ("wordpiece-30522.json", "chatbpe-32000.json"):
        f = T._ASSETS / name
        assert f.exists(), f
        json.loads(f.read_text())
    monkeypatch.setattr(T, "_CACHE", tmp_path / "none")        # no build-dir cache to fall back on
    monkeypatch.setattr(T, "_instances", {})
    monkeypatch.delenv("DOCQA_WORDPIECE_JSON", raising=False)
    trained = []
    monkeypatch.setattr(T, "_train_wordpiece", lambda v: trained.append(v))
    wp = T.WordPieceTokenizer()
    assert not trained and wp.vocab_size > 1000
    assert wp.tok.to_str() == T.Tokenizer.from_file(str(T._ASSETS / "wordpiece-30522.json")).to_str()
