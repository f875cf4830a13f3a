"""Wire contracts (pydantic) of every service -- the API-compatibility surface.

Reference sources: llm-qa/main.py:108-122 (Query / ask response),
synthese-comparative/models/requests.py:6-21 and models/responses.py:6-38,
synthese-comparative/core/llm_client.py:42-54 (summarize contract),
synthese-comparative/core/retrieval_client.py:72-91 (patient-snippets contract),
doc-ingestor/models.py:5-12 (document row), AMQP messages.
"""
from __future__ import annotations

from typing import List, Optional

from pydantic import BaseModel, Field


# ---------------------------------------------------------------- llm-qa
class Query(BaseModel):
    question: str


class AskResponse(BaseModel):
    answer: str
    sources: List[Optional[str]]


class SummarizeRequest(BaseModel):
    prompt: str


class SummarizeResponse(BaseModel):
    summary: str


# ---------------------------------------------------------------- semantic-indexer
class Snippet(BaseModel):
    doc_id: str
    text: str


class SearchHit(BaseModel):
    id: int
    score: float
    text: str
    source: Optional[str] = None
    type: Optional[str] = None
    doc_id: Optional[str] = None


class SearchRequest(BaseModel):
    query: str
    k: int = 3


# ---------------------------------------------------------------- synthese-comparative
class PatientSummaryRequest(BaseModel):
    patient_id: str
    from_date: Optional[str] = None
    to_date: Optional[str] = None
    focus: Optional[str] = None
    language: str = "fr"


class PatientComparisonRequest(BaseModel):
    patient_ids: List[str]
    from_date: Optional[str] = None
    to_date: Optional[str] = None
    focus: Optional[str] = None
    language: str = "fr"


class SourceSnippet(BaseModel):
    doc_id: str
    snippet: str


class Section(BaseModel):
    title: str
    content: str


class SinglePatientSummaryResponse(BaseModel):
    type: str = "single_patient_summary"
    patient_alias: str
    time_range: Optional[dict]
    sections: List[Section]
    key_points: List[str]
    sources: List[SourceSnippet]


class ComparisonRow(BaseModel):
    dimension: str
    patient_1: str
    patient_2: str


class MultiPatientComparisonResponse(BaseModel):
    type: str = "multi_patient_comparison"
    patients: List[str]
    time_range: Optional[dict]
    summary: str
    comparison_table: List[ComparisonRow]
    key_risks: List[str]
    sources: List[SourceSnippet]


# ---------------------------------------------------------------- doc-ingestor
class DocumentOut(BaseModel):
    id: int
    filename: Optional[str]
    upload_date: Optional[str]
    status: Optional[str]
    doc_type: Optional[str]


# ---------------------------------------------------------------- queue messages
class RawDocumentMessage(BaseModel):
    doc_id: int
    text: str
    metadata: dict = Field(default_factory=dict)


class CleanDocumentMessage(BaseModel):
    doc_id: object
    original_text_masked: str
    metadata: dict = Field(default_factory=dict)
    processed_at: float
