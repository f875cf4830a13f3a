"""synthese-comparative service (FastAPI + router at /api, port 8005).

Contract (synthese-comparative/api/routes.py:22-140, models/*.py, core/*.py):
  GET  /api/status                 -> {"status": "SyntheseComparative is running"}
  POST /api/synthese/patient       PatientSummaryRequest -> SinglePatientSummaryResponse
                                   404 "No documents found for this patient."
  POST /api/synthese/comparaison   PatientComparisonRequest -> MultiPatientComparisonResponse
                                   400 "At least two patients are required."
Clients (FAKE by default, like the reference; USE_FAKE_LLM / USE_FAKE_RETRIEVAL):
  * LLMClient: FAKE keeps the LAST ``max_chars`` (1200) characters of the prompt; REAL
    posts ``{"prompt"}`` to ``LLM_QA_URL/api/llm/summarize`` (60 s) and falls back to FAKE
    on an empty reply or any error (core/llm_client.py:19-65).
  * RetrievalClient: FAKE returns two canned notes; REAL GETs
    ``SEMANTIC_INDEXER_URL/api/search/patient-snippets`` (30 s), no fallback
    (core/retrieval_client.py:25-91).  Both endpoints exist in this framework
    (services/qa.py, services/indexer.py), so REAL mode works end to end.
Per-patient retrieval in comparisons runs concurrently (the reference awaits patients
one after another).
"""
from __future__ import annotations

import asyncio
from typing import Optional

import httpx
from fastapi import APIRouter, FastAPI, HTTPException

from ..config import Settings
from ..schemas import (ComparisonRow, MultiPatientComparisonResponse, PatientComparisonRequest,
                       PatientSummaryRequest, Section, SinglePatientSummaryResponse, SourceSnippet)

# the reference's templates, verbatim (synthese-comparative/core/prompts.py:3-45)
from ..prompts import MULTI_PATIENT_TEMPLATE, SINGLE_PATIENT_TEMPLATE  # noqa: E402


class LLMClient:
    def __init__(self, base_url: Optional[str] = None, settings: Settings | None = None):
        self.st = settings or Settings()
        self.base_url = base_url or self.st.llm_qa_url

    def summarize(self, prompt: str, max_chars: int = 1200) -> str:
        if self.st.use_fake_llm:
            return self._summarize_fake(prompt, max_chars)
        return self._summarize_remote(prompt)

    @staticmethod
    def _summarize_fake(prompt: str, max_chars: int) -> str:
        return prompt if len(prompt) <= max_chars else prompt[-max_chars:]

    def _call_llm_qa_sync(self, prompt: str) -> str:
        with httpx.Client(timeout=self.st.llm_timeout_s) as client:
            resp = client.post(f"{self.base_url}/api/llm/summarize", json={"prompt": prompt})
            resp.raise_for_status()
            return resp.json().get("summary", "")

    def _summarize_remote(self, prompt: str) -> str:
        try:
            out = self._call_llm_qa_sync(prompt)
            return out if out else self._summarize_fake(prompt, self.st.fake_max_chars)
        except Exception:  # noqa: BLE001 - never break the service on LLM failure
            return self._summarize_fake(prompt, self.st.fake_max_chars)


class RetrievalClient:
    def __init__(self, base_url: Optional[str] = None, settings: Settings | None = None):
        self.st = settings or Settings()
        self.base_url = base_url or self.st.semantic_indexer_url

    async def get_patient_documents(self, patient_id: str, from_date=None, to_date=None, focus=None) -> list[dict]:
        if self.st.use_fake_retrieval:
            return self._get_fake_documents(patient_id, from_date, to_date, focus)
        return await self._get_real_documents(patient_id, from_date, to_date, focus)

    @staticmethod
    def _get_fake_documents(patient_id, from_date, to_date, focus) -> list[dict]:
        t1 = (f"Note clinique du patient {patient_id}. Période : {from_date} -> {to_date}. "
              f"Focus : {focus or 'général'}. Traitement anticoagulant en cours, INR contrôlé "
              "régulièrement.")
        t2 = ("Événement : réduction de dose après un saignement mineur ; pas d'autre événement "
              "majeur signalé ensuite.")
        return [{"doc_id": f"FAKE-DOC-{patient_id}-1", "text": t1},
                {"doc_id": f"FAKE-DOC-{patient_id}-2", "text": t2}]

    async def _get_real_documents(self, patient_id, from_date, to_date, focus) -> list[dict]:
        params = {k: v for k, v in {"patient_id": patient_id, "from_date": from_date,
                                     "to_date": to_date, "focus": focus}.items() if v is not None}
        async with httpx.AsyncClient(timeout=self.st.retrieval_timeout_s) as client:
            resp = await client.get(f"{self.base_url}/api/search/patient-snippets", params=params)
            resp.raise_for_status()
            return resp.json()


def make_router(llm_client: LLMClient | None = None, retrieval_client: RetrievalClient | None = None,
                settings: Settings | None = None) -> APIRouter:
    st = settings or Settings()
    llm = llm_client or LLMClient(settings=st)
    ret = retrieval_client or RetrievalClient(settings=st)
    router = APIRouter()

    @router.get("/status")
    async def status():
        return {"status": "SyntheseComparative is running"}

    @router.post("/synthese/patient", response_model=SinglePatientSummaryResponse)
    async def generate_patient_summary(req: PatientSummaryRequest):
        docs = await ret.get_patient_documents(req.patient_id, req.from_date, req.to_date, req.focus)
        if not docs:
            raise HTTPException(status_code=404, detail="No documents found for this patient.")
        documents = "\n\n".join(f"[{d.get('doc_id', 'UNKNOWN')}]\n{d.get('text', '')}" for d in docs)
        prompt = SINGLE_PATIENT_TEMPLATE.format(
            patient_alias=f"PATIENT_{req.patient_id}", from_date=req.from_date or "N/A",
            to_date=req.to_date or "N/A", focus=req.focus or "général", documents=documents)
        summary = await asyncio.to_thread(llm.summarize, prompt)
        return SinglePatientSummaryResponse(
            patient_alias=f"PATIENT_{req.patient_id}",
            time_range={"from": req.from_date, "to": req.to_date},
            sections=[Section(title="Synthèse clinique", content=summary)],
            key_points=[],
            sources=[SourceSnippet(doc_id=d.get("doc_id", "UNKNOWN"), snippet=d.get("text", "")[:300])
                     for d in docs[:5]])

    @router.post("/synthese/comparaison", response_model=MultiPatientComparisonResponse)
    async def generate_patient_comparison(req: PatientComparisonRequest):
        if len(req.patient_ids) < 2:
            raise HTTPException(status_code=400, detail="At least two patients are required.")
        per_patient = await asyncio.gather(*[
            ret.get_patient_documents(pid, req.from_date, req.to_date, req.focus) for pid in req.patient_ids])
        text, sources = "", []
        for pid, docs in zip(req.patient_ids, per_patient):
            text += f"\n\n=== PATIENT_{pid} ===\n"
            for d in docs:
                text += f"[{d.get('doc_id', 'UNKNOWN')}]\n{d.get('text', '')}\n"
            sources += [SourceSnippet(doc_id=d.get("doc_id", "UNKNOWN"), snippet=d.get("text", "")[:300])
                        for d in docs[:3]]
        aliases = [f"PATIENT_{p}" for p in req.patient_ids]
        prompt = MULTI_PATIENT_TEMPLATE.format(
            patients=aliases, from_date=req.from_date or "N/A", to_date=req.to_date or "N/A",
            focus=req.focus or "général", documents_by_patient=text)
        summary = await asyncio.to_thread(llm.summarize, prompt)
        table = [ComparisonRow(dimension="Exemple de dimension",
                               patient_1="Informations principales patient 1",
                               patient_2="Informations principales patient 2")]
        return MultiPatientComparisonResponse(
            patients=aliases, time_range={"from": req.from_date, "to": req.to_date}, summary=summary,
            comparison_table=table, key_risks=[], sources=sources[:10])

    return router


def create_app(settings: Settings | None = None, llm_client=None, retrieval_client=None) -> FastAPI:
    app = FastAPI(title="SyntheseComparative Microservice (MI355X)", version="1.0.0")
    app.include_router(make_router(llm_client, retrieval_client, settings), prefix="/api", tags=["synthese"])
    return app
