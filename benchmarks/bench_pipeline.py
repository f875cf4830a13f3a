"""BASELINE.json config 5: the full pipeline -- ingest -> de-identify -> embed -> retrieve
-> Llama-3-70B generate, tensor-parallel over the GPUs of one node (RCCL / xGMI), the
vector index sharded across every GPU.

Launch: ``torchrun --nproc-per-node N --master-addr 127.0.0.1 benchmarks/bench_pipeline.py``
(TP = N by default; ``--tp`` for TP x DP mixes).  On one MI355X it runs the same path at
TP=1 (Llama-3-70B bf16 is 141 GB: it fits in 288 GB of HBM with its KV cache).

Stage 1 (ingest, timed): each rank takes every world-th synthetic clinical note, runs the
deid-service path (clinical-BERT NER token classifier on the HIP encoder kernels +
pattern/context recognizers + ``<ENTITY>`` replacement, one packed batch per burst), the
semantic-indexer path (500-char chunks, "Dossier Patient {id}" sources, MiniLM embed on
the HIP kernels) and adds the chunks to its local shard of the flat L2 index.
Stage 2 (QA, timed): batches of questions -> query embed -> sharded kNN (each GPU scans
its shard with the fused MFMA distance + top-k kernel; the per-shard top-k is merged with
one all-gather on a dedicated process group) -> RAG prompt -> TP generation (column /
row-parallel projections, the IPC all-reduce with residual + RMSNorm fused (RCCL when IPC
mapping is unavailable), HIP-graph decode).
Synthetic notes + random-init weights of the named architectures.  Rank 0 prints one
JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--llm", default="llama3-70b")
    ap.add_argument("--embed", default="minilm-l6")
    ap.add_argument("--ner", default="clinical-bert")
    ap.add_argument("--tp", type=int, default=0, help="tensor-parallel size (default: world size)")
    ap.add_argument("--notes", type=int, default=2000)
    ap.add_argument("--burst", type=int, default=64, help="notes per de-identification / embed burst")
    ap.add_argument("--batch", type=int, default=64, help="questions per step")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--max-new-tokens", type=int, default=128)
    ap.add_argument("--max-context", type=int, default=2048)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--kv-mem-fraction", type=float, default=0.85,
                    help="KV pool = this fraction of the HBM free after the weights (0: max_batch full contexts)")
    ap.add_argument("--pipelined", action="store_true",
                    help="overlap batch i+1's embed/search with batch i's decode tail")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--share-gpu", action="store_true",
                    help="every rank on cuda:0: a one-GPU rehearsal of the TP=N path (gloo process group, "
                         "IPC all-reduce between the ranks' processes); correctness, not speed")
    ap.add_argument("--questions", choices=("unique", "repeat"), default="unique",
                    help="unique: every request a distinct question; repeat: the small template grid")
    a = ap.parse_args()

    import torch
    import torch.distributed as dist

    from docqa_amd import ops
    from docqa_amd.deid.engine import NER_LABELS, DeidEngine
    from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
    from docqa_amd.index.flat import FlatIndex
    from docqa_amd.index.sharded import ShardedFlatIndex
    from docqa_amd.models.bert import BertConfig, BertTokenClassifier
    from docqa_amd.models import checkpoint as ck
    from docqa_amd.parallel import comm
    from docqa_amd.pipeline.corpus import embed_records
    from docqa_amd.pipeline.rag import RAGPipeline
    from docqa_amd.text.chunking import chunk_chars
    from docqa_amd.text.kb import synthetic_kb_records
    from docqa_amd.text.synthetic import synthetic_notes, synthetic_questions, synthetic_unique_questions
    from docqa_amd.text.tokenizer import ChatTokenizer, WordPieceTokenizer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    tp = a.tp or world
    cuda = a.device == "cuda"
    local_rank = 0 if a.share_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    if cuda:
        torch.cuda.set_device(local_rank)
    ps = comm.init_distributed(tp_size=tp, backend="gloo" if (a.share_gpu or not cuda) else None)
    if cuda and a.share_gpu and tp > 1:
        comm.enable_custom_all_reduce(force=True)
    if cuda:
        assert ops.load_native(), "native HIP kernels not built (python -m docqa_amd.ops.build)"
    dev = f"cuda:{local_rank}" if cuda else "cpu"
    # the index gets its own communicator: its all-gathers never interleave with the TP
    # all-reduces of the generator on one communicator
    idx_group = dist.new_group(list(range(ps.world_size))) if ps.world_size > 1 else None

    def sync():
        if cuda:
            torch.cuda.synchronize()

    t_setup = time.perf_counter()

    def note(msg: str) -> None:     # progress on stderr (rank 0): long TP rehearsals stay visibly alive
        if ps.rank == 0:
            print(f"[bench_pipeline] {msg} ({time.perf_counter() - t_setup:.0f} s)", file=sys.stderr, flush=True)

    def tmax(x: float) -> float:
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        if dist.is_initialized():
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    enc_tok = WordPieceTokenizer()
    ner_tok = WordPieceTokenizer(max_len=256)
    encoder = ck.resolve_bert(a.embed, device=dev, seed=0)        # preset or checkpoint dir
    ner = (ck.load_bert_token_classifier(a.ner, NER_LABELS, device=dev) if ck.is_checkpoint(a.ner)
           else BertTokenClassifier(BertConfig.preset(a.ner), NER_LABELS, device=dev))
    deid = DeidEngine(ner, ner_tok, use_model=True)
    local = FlatIndex(encoder.cfg.hidden, "l2", dev, capacity=1 << 16)
    # knowledge-base bootstrap (semantic-indexer startup), sharded across the ranks
    kb = synthetic_kb_records()
    records = kb[ps.rank::ps.world_size]
    local.add(embed_records(encoder, enc_tok, records))

    note("encoders and KB index ready")
    # ---------------------------------------------------------------- stage 1: ingest
    notes = synthetic_notes(a.notes, seed=11)
    mine = list(range(ps.rank, len(notes), ps.world_size))
    warm = [n["text"] for n in notes[:4]]
    deid.process_batch(warm)                              # warm the NER / encoder kernels
    embed_records(encoder, enc_tok, [{"text_content": t} for t in warm])
    sync()
    comm.barrier()
    t0 = time.perf_counter()
    n_chunks = 0
    for i in range(0, len(mine), a.burst):
        ids = mine[i:i + a.burst]
        clean = deid.process_batch([notes[j]["text"] for j in ids])
        recs = []
        for j, text in zip(ids, clean):
            for c in chunk_chars(text, 500):
                recs.append({"doc_id": str(j + 1), "text_content": c, "source": f"Dossier Patient {j + 1}",
                             "type": "patient_file", "patient_id": notes[j].get("patient_id", str(j + 1))})
        if recs:
            local.add(embed_records(encoder, enc_tok, recs))
            records.extend(recs)
            n_chunks += len(recs)
    sync()
    t_ingest = tmax(time.perf_counter() - t0)
    if dist.is_initialized():
        cnt = torch.tensor([n_chunks], dtype=torch.long, device=dev)
        dist.all_reduce(cnt)
        tot_chunks = int(cnt)
    else:
        tot_chunks = n_chunks

    # global metadata in shard order (ids = shard offset + local row)
    if dist.is_initialized():
        parts = [None] * ps.world_size
        dist.all_gather_object(parts, records, group=idx_group)
        all_records = [r for p in parts for r in p]
        index = ShardedFlatIndex(local, group=idx_group, replicated=ps.dp_size == 1)
    else:
        all_records, index = records, local

    note(f"ingested {tot_chunks} chunks")
    # ---------------------------------------------------------------- stage 2: QA
    model = ck.resolve_llama(a.llm, device=dev, seed=0)
    note(f"{a.llm} shard built (TP {tp})")
    llm_cfg = model.cfg
    # KV pool from the HBM left after the weights (the Llama-3-70B weights alone are 141 GB:
    # max_batch full contexts no longer fit beside them at batch 256)
    engine = LLMEngine(model, max_batch=a.batch, max_context=a.max_context, use_graphs=cuda,
                       kv_mem_fraction=(a.kv_mem_fraction or None) if cuda else None)
    chat_tok = ChatTokenizer(model_vocab=llm_cfg.vocab_size)
    pipe = RAGPipeline(encoder, enc_tok, index, all_records, engine, chat_tok, k=a.k,
                       max_prompt_tokens=a.max_context - a.max_new_tokens - 64)
    sync()
    setup_s = tmax(time.perf_counter() - t_setup)
    params = SamplingParams(max_new_tokens=a.max_new_tokens, temperature=0.0, stop_on_eos=False)
    gen_q = synthetic_unique_questions if a.questions == "unique" else synthetic_questions
    qs = gen_q((a.warmup + a.steps) * ps.dp_size * a.batch, seed=321)

    def batch_for(step: int) -> list[str]:
        base = (step * ps.dp_size + ps.dp_rank) * a.batch
        return qs[base:base + a.batch]

    def run(steps: list[int]) -> list[float]:
        lat = []
        if a.pipelined:
            for _, _, l in pipe.answer_pipelined([batch_for(s) for s in steps], params):
                lat.append(l)
        else:
            for s in steps:
                t = time.perf_counter()
                pipe.answer_batch(batch_for(s), params)
                sync()
                lat.append(time.perf_counter() - t)
        return lat

    run(list(range(a.warmup)))
    sync()
    note("warm-up done")
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    lat = run(list(range(a.warmup, a.warmup + a.steps)))
    sync()
    comm.barrier()
    sync()
    elapsed = tmax(time.perf_counter() - t0)
    lat = [tmax(x) for x in lat]
    queries = ps.dp_size * a.batch * a.steps
    if ps.rank == 0:
        out = {
            "metric": "pipeline_e2e_qa_queries_per_sec",
            "value": round(queries / elapsed, 3),
            "unit": "queries/s",
            "n_gpus": ps.world_size,
            "p50_latency_ms": round(1e3 * statistics.median(lat), 1),
            "ingest_docs_per_sec": round(len(notes) / t_ingest, 1),
            "ingest_chunks_per_sec": round(tot_chunks / t_ingest, 1),
            "ingest_s": round(t_ingest, 2),
            "gen_tokens_per_sec": round(queries * a.max_new_tokens / elapsed, 1),
            "dtype": "bf16",
            "data": "synthetic clinical notes + questions, random-init weights",
            "config": {"config": "BASELINE config 5", "llm": a.llm, "embed": a.embed, "ner": a.ner,
                       "parallelism": f"tp{tp}" + (f"xdp{ps.dp_size}" if ps.dp_size > 1 else ""),
                       "index": f"flat-L2 sharded x{ps.world_size}", "index_vectors": len(all_records),
                       "notes": len(notes), "batch": a.batch, "max_new_tokens": a.max_new_tokens,
                       "k": a.k, "pipelined": a.pipelined, "questions": a.questions,
                       "tp_all_reduce": "ipc-fused" if comm.custom_all_reduce() is not None else
                                        ("rccl" if tp > 1 and cuda else ("gloo" if tp > 1 else "none"))},
            "setup_s": round(setup_s, 1),
            "prefix_cached_frac": round(engine.stats.cached_tokens / max(1, engine.stats.prompt_tokens), 3),
        }
        print(json.dumps(out), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
