"""Environment-variable configuration.

Names and defaults follow the reference so existing deployments keep
working; the hard-coded constants of the reference are exposed as variables too, plus
the MI355X knobs of this framework.

| variable | default | reference site |
|---|---|---|
| RABBITMQ_HOST | localhost | doc-ingestor/processing.py:7, deid-service/anonymizer.py:20 |
| DB_HOST / DB_PORT | localhost / 5433 | doc-ingestor/database.py:7-8 |
| INPUT_QUEUE / OUTPUT_QUEUE | raw_documents_queue / clean_documents_queue | deid-service/anonymizer.py:21-22 |
| NLP_LANG | en | deid-service/anonymizer.py:24 |
| OLLAMA_BASE_URL | http://localhost:11434 | llm-qa/main.py:66 (unused: generation is in-process) |
| SEMANTIC_INDEXER_URL | http://semantic-indexer:8003 | synthese-comparative/core/config.py:10-13 |
| LLM_QA_URL | http://llm-qa:8004 | synthese-comparative/core/config.py:16-19 |
| USE_FAKE_RETRIEVAL / USE_FAKE_LLM | true / true | synthese-comparative/core/config.py:22-23 |
| DEID_NER | auto | the spaCy NER of deid-service/anonymizer.py:29,41-45: "auto" runs the token classifier -- NER_CHECKPOINT's, else the shipped synthetic-trained one (deid/assets/ner-synthetic) --, "1" always, "0" never |
| NER_CHECKPOINT | (empty) | Hugging Face BERT token-classification checkpoint directory for DEID_NER |
| DEID_BATCH_DOCS | 32 | raw messages the deid worker drains into one packed NER forward |
| MAX_BATCH | 256 on a GPU, 64 on CPU | llm-qa decode slots (the measured batch) |
| MAX_CONTEXT | 8192 | llm-qa engine context (prompt + generation); Llama-3's window |
| QA_TEMPLATE | reference | llm-qa prompt: the verbatim reference text (llm-qa/main.py:71-93) or cache_friendly |
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field


def env_bool(name: str, default: str = "true") -> bool:
    """The reference's ``_env_bool``: "1/true/yes/y" (case-insensitive) are true."""
    return os.getenv(name, default).lower() in ("1", "true", "yes", "y")


def env_int(name: str, default: int) -> int:
    try:
        return int(os.getenv(name, str(default)))
    except ValueError:
        return default


@dataclass
class Settings:
    # transport / infra (reference names)
    rabbitmq_host: str = field(default_factory=lambda: os.getenv("RABBITMQ_HOST", "localhost"))
    bus_backend: str = field(default_factory=lambda: os.getenv("DOCQA_BUS", "inproc"))  # inproc | spool | amqp
    bus_journal_dir: str = field(default_factory=lambda: os.getenv("DOCQA_BUS_JOURNAL", ""))
    spool_dir: str = field(default_factory=lambda: os.getenv("DOCQA_SPOOL_DIR", "docqa_spool"))  # DOCQA_BUS=spool
    db_host: str = field(default_factory=lambda: os.getenv("DB_HOST", "localhost"))
    db_port: str = field(default_factory=lambda: os.getenv("DB_PORT", "5433"))
    database_url: str = field(default_factory=lambda: os.getenv("DATABASE_URL", "sqlite:///docqa_documents.db"))
    raw_queue: str = field(default_factory=lambda: os.getenv("INPUT_QUEUE", "raw_documents_queue"))
    clean_queue: str = field(default_factory=lambda: os.getenv("OUTPUT_QUEUE", "clean_documents_queue"))
    nlp_lang: str = field(default_factory=lambda: os.getenv("NLP_LANG", "en"))
    # de-identification: NER token classifier in the loop (auto: when a checkpoint is set)
    deid_ner: str = field(default_factory=lambda: os.getenv("DEID_NER", "auto").lower())
    ner_checkpoint: str = field(default_factory=lambda: os.getenv("NER_CHECKPOINT", ""))
    deid_batch_docs: int = field(default_factory=lambda: env_int("DEID_BATCH_DOCS", 32))
    tika_url: str = field(default_factory=lambda: os.getenv("TIKA_URL", ""))  # empty: native extractors
    upload_dir: str = field(default_factory=lambda: os.getenv("UPLOAD_DIR", "temp_uploads"))
    # indexer
    index_dir: str = field(default_factory=lambda: os.getenv("INDEX_DIR", "."))
    index_file: str = field(default_factory=lambda: os.getenv("INDEX_FILE", "vector_store.faiss"))
    metadata_file: str = field(default_factory=lambda: os.getenv("METADATA_FILE", "metadata_store.pkl"))
    # durability: every indexed batch is appended to <index>.wal (O(batch) bytes); the
    # FAISS + pickle snapshot pair is rewritten every INDEX_SNAPSHOT_EVERY batches
    index_wal: bool = field(default_factory=lambda: env_bool("INDEX_WAL", "true"))
    snapshot_every: int = field(default_factory=lambda: env_int("INDEX_SNAPSHOT_EVERY", 16))
    default_data_dir: str = field(default_factory=lambda: os.getenv("DEFAULT_DATA_DIR", "default_data"))
    chunk_size: int = field(default_factory=lambda: env_int("CHUNK_SIZE", 500))
    # vector store: flat (IndexFlatL2, the reference's) | ivfpq (IndexRefineFlat over IVF-PQ,
    # trained once IVF_TRAIN_MIN vectors are stored -- index/hybrid.py)
    index_type: str = field(default_factory=lambda: os.getenv("INDEX_TYPE", "flat"))
    ivf_nlist: int = field(default_factory=lambda: env_int("IVF_NLIST", 1024))
    pq_m: int = field(default_factory=lambda: env_int("PQ_M", 0))                 # 0: d / 8
    ivf_nprobe: int = field(default_factory=lambda: env_int("IVF_NPROBE", 32))
    # exact re-rank of min(64, k x REFINE_K_FACTOR) IVF-PQ candidates (k = 3 for the QA
    # retriever: 48 candidates)
    refine_k_factor: int = field(default_factory=lambda: env_int("REFINE_K_FACTOR", 16))
    # orthogonal PQ pre-rotation: pca (principal directions dealt round-robin to the
    # sub-quantizers; FAISS IndexPreTransform) | none
    pq_rotation: str = field(default_factory=lambda: os.environ.get("PQ_ROTATION", "pca"))
    ivf_train_min: int = field(default_factory=lambda: env_int("IVF_TRAIN_MIN", 0))  # 0: 39 x nlist
    embed_model: str = field(default_factory=lambda: os.getenv("EMBED_MODEL", "minilm-l6"))
    # llm-qa
    llm_model: str = field(default_factory=lambda: os.getenv("LLM_MODEL", "llama3-8b"))
    top_k: int = field(default_factory=lambda: env_int("TOP_K", 3))
    max_new_tokens: int = field(default_factory=lambda: env_int("MAX_NEW_TOKENS", 256))
    temperature: float = field(default_factory=lambda: float(os.getenv("TEMPERATURE", "0")))
    # stop a generation at EOS (the reference's behaviour); STOP_ON_EOS=0 decodes every
    # answer to MAX_NEW_TOKENS (serving benchmarks: random weights emit EOS at random)
    stop_on_eos: bool = field(default_factory=lambda: env_bool("STOP_ON_EOS", "true"))
    # decode slots: MAX_BATCH, else 256 on a GPU -- the batch every throughput number in
    # profiles/ and BENCH_r*.json is measured at -- and 64 on CPU
    max_batch: int = field(default_factory=lambda: _default_max_batch())
    # engine context window (prompt + generation): long synthese prompts are prefilled in
    # chunks up to it and truncated only beyond it
    max_context: int = field(default_factory=lambda: env_int("MAX_CONTEXT", 8192))
    batch_window_ms: int = field(default_factory=lambda: env_int("BATCH_WINDOW_MS", 5))
    # llm-qa scheduling: "continuous" (requests join/leave the decode batch every step,
    # engine/scheduler.py) or "batch" (static batches, one prefill + decode loop each)
    serving_mode: str = field(default_factory=lambda: os.getenv("DOCQA_SERVING", "continuous"))
    tp_size: int = field(default_factory=lambda: env_int("TP_SIZE", 1))
    device: str = field(default_factory=lambda: os.getenv("DOCQA_DEVICE", "auto"))
    # synthese
    semantic_indexer_url: str = field(default_factory=lambda: os.getenv("SEMANTIC_INDEXER_URL", "http://semantic-indexer:8003"))
    llm_qa_url: str = field(default_factory=lambda: os.getenv("LLM_QA_URL", "http://llm-qa:8004"))
    # clinical UI back ends (the reference UI's hard-coded localhost ports; containers set
    # the service names, deploy/docker-compose.yml)
    ui_ingest_url: str = field(default_factory=lambda: os.getenv("DOC_INGESTOR_URL", "http://127.0.0.1:8000"))
    ui_qa_url: str = field(default_factory=lambda: os.getenv("UI_LLM_QA_URL", "http://127.0.0.1:8001"))
    use_fake_retrieval: bool = field(default_factory=lambda: env_bool("USE_FAKE_RETRIEVAL", "true"))
    use_fake_llm: bool = field(default_factory=lambda: env_bool("USE_FAKE_LLM", "true"))
    fake_max_chars: int = 1200
    llm_timeout_s: float = 60.0
    retrieval_timeout_s: float = 30.0

    def ner_enabled(self) -> bool:
        """Whether the deid worker runs the NER model (DEID_NER auto / 1 / 0)."""
        if self.deid_ner in ("1", "true", "yes", "y", "on"):
            return True
        if self.deid_ner in ("0", "false", "no", "n", "off"):
            return False
        from .deid.engine import shipped_ner

        return bool(self.ner_checkpoint) or shipped_ner() is not None

    def ner_source(self, fallback: str) -> str:
        """The NER model to load: NER_CHECKPOINT, else the shipped synthetic-trained
        checkpoint (deid/assets/ner-synthetic), else ``fallback`` (a random-init preset)."""
        if self.ner_checkpoint:
            return self.ner_checkpoint
        from .deid.engine import shipped_ner

        return shipped_ner() or fallback

    def resolved_device(self) -> str:
        if self.device != "auto":
            return self.device
        try:
            import torch

            return "cuda" if torch.cuda.is_available() else "cpu"
        except Exception:
            return "cpu"


def default_max_batch(device: str | None = None) -> int:
    """MAX_BATCH, else by device: 256 decode slots on a GPU, 64 on the CPU.  ``device``:
    the device the engine will run on (``StackOptions.device``); None reads DOCQA_DEVICE,
    and ``auto`` looks for the GPU driver node WITHOUT initialising the HIP runtime (a
    settings read in a CPU-only service process must not start it -- ADVICE r5)."""
    if os.environ.get("MAX_BATCH"):
        return env_int("MAX_BATCH", 256)
    dev = device if device is not None else os.environ.get("DOCQA_DEVICE", "auto")
    if dev == "auto":
        dev = "cuda" if os.path.exists("/dev/kfd") else "cpu"
    return 256 if str(dev).startswith("cuda") else 64


def _default_max_batch() -> int:
    return default_max_batch()


def settings() -> Settings:
    return Settings()
