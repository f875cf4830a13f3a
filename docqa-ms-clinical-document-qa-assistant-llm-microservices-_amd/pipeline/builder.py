"""Assemble the QA stack (encoder + index + generator) for services, bench and smoke."""
from __future__ import annotations

import os
import time
from dataclasses import dataclass

import torch

from ..engine.llm_engine import LLMEngine
from ..index.flat import FlatIndex
from ..index.sharded import ShardedFlatIndex
from ..models import checkpoint as ck
from ..parallel import comm
from ..text.tokenizer import ChatTokenizer, WordPieceTokenizer
from .corpus import build_corpus, embed_records
from .rag import RAGPipeline


@dataclass
class StackConfig:
    llm: str = "llama3-8b"
    embed: str = "minilm-l6"
    n_notes: int = 1000
    kb_dir: str | None = None
    max_batch: int = 64
    max_context: int = 2048
    k: int = 3
    storage_dtype: torch.dtype = torch.float32
    use_graphs: bool = True
    seed: int = 0
    kv_mem_fraction: float | None = None   # size the KV pool from free HBM (LLMEngine)


def build_stack(sc: StackConfig, device="cuda", log=print) -> tuple[RAGPipeline, dict]:
    info = {}
    t0 = time.perf_counter()
    s = comm.state()
    # names are presets (random-init weights) or Hugging Face checkpoint directories
    ck.use_checkpoint_tokenizers(sc.llm, sc.embed)
    llm_cfg = ck.resolve_llama_config(sc.llm)
    enc_tok = WordPieceTokenizer()
    chat_tok = ChatTokenizer(model_vocab=llm_cfg.vocab_size)
    encoder = ck.resolve_bert(sc.embed, device=device, seed=sc.seed)
    records = build_corpus(sc.n_notes, sc.kb_dir, sc.seed)
    # contiguous shard per data-parallel rank: global ids = shard offset + local row
    n = len(records)
    lo = n * s.dp_rank // s.dp_size
    hi = n * (s.dp_rank + 1) // s.dp_size
    emb = embed_records(encoder, enc_tok, records[lo:hi])
    local = FlatIndex(encoder.cfg.hidden, "l2", device, sc.storage_dtype, capacity=max(1024, hi - lo))
    local.add(emb)
    # queries padded to the static batch size: no per-search count exchange / host sync
    index = ShardedFlatIndex(local, max_queries=sc.max_batch) if s.dp_size > 1 else local
    if s.dp_size > 1 and os.environ.get("DOCQA_SHARD_IPC", "1") == "1":
        # per-batch query / top-k all-gathers on the IPC peer-memory kernel (off RCCL)
        index.enable_ipc()
    if device != "cpu" and torch.device(device).type == "cuda":
        torch.cuda.synchronize()
    info["index_build_s"] = time.perf_counter() - t0
    info["index_vectors"] = n
    model = ck.resolve_llama(sc.llm, device=device, seed=sc.seed)
    engine = LLMEngine(model, max_batch=sc.max_batch, max_context=sc.max_context,
                       use_graphs=sc.use_graphs, kv_mem_fraction=sc.kv_mem_fraction)
    info["kv_blocks"] = engine.kv.allocator.num_blocks if hasattr(engine.kv.allocator, "num_blocks") else None
    pipe = RAGPipeline(encoder, enc_tok, index, records, engine, chat_tok, k=sc.k,
                       max_prompt_tokens=sc.max_context - 256)
    if s.dp_size > 1:
        # every rank has finished its (seconds-long, rank-skewed) weight init and KV pool
        # before any rank enters the first search: the shard gathers start aligned
        if device != "cpu" and torch.device(device).type == "cuda":
            torch.cuda.synchronize()
        comm.barrier()
    info["setup_s"] = time.perf_counter() - t0
    return pipe, info
