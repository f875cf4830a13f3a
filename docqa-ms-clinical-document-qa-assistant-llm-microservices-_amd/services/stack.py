"""The whole DocQA stack in one process (one MI355X, or CPU with tiny models).

Wiring (SURVEY.md §1 data flow, with the process boundaries that carried no compute
removed): doc-ingestor -> bus(raw_documents_queue) -> deid worker (NER on the GPU) ->
bus(clean_documents_queue) -> semantic indexer (encoder + HBM index) -> the llm-qa RAG
pipeline shares the *live* index object, so a document is answerable as soon as its
status turns INDEXED.  synthese-comparative is wired in REAL mode to the in-process
retrieval and LLM when ``real_synthese`` is set.  ``launch.py`` serves each app on the
reference's port.
"""
from __future__ import annotations

import logging
import tempfile
from dataclasses import dataclass, field

from ..bus.broker import InProcBroker, get_broker
from ..index.follower import IndexFollower
from ..config import Settings
from ..deid.engine import NER_LABELS, DeidEngine
from ..engine.llm_engine import LLMEngine
from ..models import checkpoint as ck
from ..models.bert import BertConfig, BertTokenClassifier
from ..pipeline.rag import RAGPipeline
from ..store import docs_db
from ..text.tokenizer import ChatTokenizer, WordPieceTokenizer
from . import deid_worker, indexer as indexer_mod, ingest, qa, synthese, ui

log = logging.getLogger("docqa.stack")


@dataclass
class StackOptions:
    llm: str = "llama3-8b"
    embed: str = "minilm-l6"
    ner: str = "clinical-bert"
    device: str = "cuda"
    max_batch: int | None = None     # None: MAX_BATCH, else 256 on a GPU / 64 on the CPU (this device)
    max_context: int | None = None   # None: Settings.max_context (MAX_CONTEXT, 8192) capped by the model
    use_graphs: bool = True
    # NER token classifier inside de-identification (reference: spaCy NER on every message,
    # deid-service/anonymizer.py:29,41-45); None: Settings.ner_enabled() (DEID_NER / NER_CHECKPOINT)
    ner_in_loop: bool | None = None
    real_synthese: bool = False
    services: tuple = ()          # subset of ALL_SERVICES hosted by this process (empty: all)
    qa_lockstep: object = None    # llm-qa leads a tensor-parallel group (services/launch.py --tp)
    qa_replicas: tuple = ()       # llm-qa front-end over these data-parallel replica URLs
    kv_mem_fraction: float | None = 0.8   # KV pool from free HBM (GPU only; LLMEngine)
    preload_notes: int = 0        # index this many synthetic clinical notes at start (benchmarks / demos)

    def __post_init__(self):
        if self.max_batch is None:
            from ..config import default_max_batch

            self.max_batch = default_max_batch(self.device)


class _LocalRetrieval(synthese.RetrievalClient):
    def __init__(self, idx, st):
        super().__init__(settings=st)
        self.idx = idx

    async def get_patient_documents(self, patient_id, from_date=None, to_date=None, focus=None):
        return self.idx.patient_snippets(patient_id, from_date, to_date, focus)


class _LocalLLM(synthese.LLMClient):
    def __init__(self, batcher, st):
        super().__init__(settings=st)
        self.batcher = batcher

    def summarize(self, prompt: str, max_chars: int = 1200) -> str:
        try:
            out = self.batcher.submit("summarize", prompt).result(timeout=self.st.llm_timeout_s)["summary"]
            return out or self._summarize_fake(prompt, max_chars)
        except Exception:  # noqa: BLE001 - same fallback as the HTTP client
            return self._summarize_fake(prompt, max_chars)


ALL_SERVICES = ("ingest", "deid", "indexer", "qa", "synthese", "ui")


class DocQAStack:
    """Build the services named in ``opts.services`` (default: all, in one process).

    Several processes can each host a subset -- the reference's deployment of one
    process per service (start_all.bat) -- when the bus crosses processes
    (``DOCQA_BUS=spool`` or ``amqp``), the documents DB is a shared URL (SQLite file or
    Postgres), and the indexer directory is shared: a llm-qa process without the
    indexer follows the indexer's snapshot + write-ahead log (index/follower.py) instead
    of holding the live index object."""

    def __init__(self, opts: StackOptions, settings: Settings | None = None):
        self.opts = opts
        self.st = settings or Settings()
        svc = set(opts.services or ALL_SERVICES)
        unknown = svc - set(ALL_SERVICES)
        if unknown:
            raise ValueError(f"unknown services {sorted(unknown)}")
        self.services = svc
        if not self.st.upload_dir or self.st.upload_dir == "temp_uploads":
            self.st.upload_dir = tempfile.mkdtemp(prefix="docqa_uploads_")
        dev = opts.device
        self.broker = (get_broker(self.st) if self.st.bus_backend != "inproc"
                       else InProcBroker(self.st.bus_journal_dir or None))
        self.db = docs_db.DocsDB(self.st.database_url) if svc & {"ingest", "indexer"} else None
        ck.use_checkpoint_tokenizers(opts.llm, opts.embed)
        self.enc_tok = WordPieceTokenizer()
        llm_cfg = ck.resolve_llama_config(opts.llm)
        self.chat_tok = ChatTokenizer(model_vocab=llm_cfg.vocab_size)
        self.encoder = ck.resolve_bert(opts.embed, device=dev) if svc & {"indexer", "qa"} else None
        self.deid = self.indexer = self.follower = self.engine = self.pipeline = None
        self.ingest_app = self.qa_app = self.indexer_app = self.synthese_app = self.ui_app = None
        if "deid" in svc:
            ner_model = None
            use_ner = self.st.ner_enabled() if opts.ner_in_loop is None else opts.ner_in_loop
            if use_ner:
                src = self.st.ner_source(opts.ner)
                ner_model = (ck.load_bert_token_classifier(src, NER_LABELS, device=dev)
                             if ck.is_checkpoint(src)
                             else BertTokenClassifier(BertConfig.preset(src), NER_LABELS, device=dev))
                log.info("deid: NER token classifier %s in the loop (batches of <= %d docs)", src,
                         self.st.deid_batch_docs)
            self.deid_engine = DeidEngine(ner_model, self.enc_tok, use_model=use_ner)
            self.deid = deid_worker.DeidWorker(self.deid_engine, self.st, self.broker).start()
        if "indexer" in svc:
            db = self.db
            self.indexer = indexer_mod.SemanticIndexer(
                self.encoder, self.enc_tok, self.st, device=dev,
                on_indexed=lambda i: db.set_status(i, docs_db.STATUS_INDEXED)).startup()
            if opts.preload_notes:
                from ..pipeline.corpus import build_corpus

                self.indexer.add_records(build_corpus(opts.preload_notes, None, 0))
                self.indexer.commit()
            self.indexer.start_consumer(self.broker)
            self.indexer_app = indexer_mod.create_app(self.indexer)
        if "qa" in svc:
            if self.indexer is not None:
                index, metadata = self.indexer.index, self.indexer.metadata
            else:
                self.follower = IndexFollower(self.st.index_dir, self.st.index_file, self.st.metadata_file,
                                              d=self.encoder.cfg.hidden, device=dev, settings=self.st).start()
                index, metadata = self.follower.index, self.follower.metadata
            self.model = ck.resolve_llama(opts.llm, device=dev)
            ctx = min(opts.max_context or self.st.max_context, self.model.cfg.max_position)
            self.engine = LLMEngine(self.model, max_batch=opts.max_batch, max_context=ctx,
                                    use_graphs=opts.use_graphs, kv_mem_fraction=opts.kv_mem_fraction)
            self.pipeline = RAGPipeline(self.encoder, self.enc_tok, index, metadata,
                                        self.engine, self.chat_tok, k=self.st.top_k,
                                        max_prompt_tokens=ctx - self.st.max_new_tokens - 8)
            self.qa_app = qa.create_app(self.pipeline, self.st, lockstep=opts.qa_lockstep,
                                        replicas=list(opts.qa_replicas) or None)
        if "ingest" in svc:
            self.ingest_app = ingest.create_app(self.st, self.db, self.broker)
        if "synthese" in svc:
            if opts.real_synthese and self.qa_app is not None and self.indexer is not None:
                self.synthese_app = synthese.create_app(
                    self.st, _LocalLLM(self.qa_app.state.batcher, self.st), _LocalRetrieval(self.indexer, self.st))
            else:   # FAKE / REAL-over-HTTP per USE_FAKE_* and the service URLs (reference behaviour)
                self.synthese_app = synthese.create_app(self.st)
        if "ui" in svc:
            self.ui_app = ui.create_app(self.st.ui_ingest_url, self.st.ui_qa_url)

    def close(self) -> None:
        if self.deid is not None:
            self.deid.stop()
        if self.indexer is not None:
            self.indexer.stop_consumer()
        if self.follower is not None:
            self.follower.stop()
        if self.qa_app is not None and self.qa_app.state.batcher is not None:
            self.qa_app.state.batcher.stop()
