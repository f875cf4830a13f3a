"""Headline benchmark: end-to-end RAG QA throughput (embed + kNN + generate) and p50
answer latency with a Llama-3-8B generator (BASELINE.json metric / config 4, scaled
data-parallel over 1-8 MI355X with the vector index sharded across the GPUs).

One step = one batch of ``--batch`` clinical questions per data-parallel rank, pushed
through the whole llm-qa path: WordPiece tokenise -> MiniLM-L6 embed (HIP encoder
kernels) -> kNN top-3 over the sharded flat L2 index (HIP MFMA distance+top-k, RCCL
all-gathers across ranks) -> stuff prompt -> Llama-3-8B bf16 prefill + greedy decode
of ``--max-new-tokens`` tokens (hand-written HIP GEMM / attention / norm / rope kernels,
HIP-graph decode loop) -> detokenise.  Synthetic clinical notes + random-init weights
of the named architectures (no checkpoints or datasets are reachable).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (N>1: launched by torchrun, one rank per GPU, RANK/WORLD_SIZE from the env)
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
# Measured reference-equivalent stack on the same MI355X (HF transformers
# Llama-3-8B batch-1 generate + eager MiniLM + exact L2, serial requests, same inputs).
REF_EQUIV_QPS = 0.6149
sys.path.insert(0, str(ROOT))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
# kernel arguments in device memory: +0.3-0.5 % on the decode loop's ~330 launches per step
# (profiles/r2_ab_dev_kernarg.log); read by the HIP runtime at init, so set before torch
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
if "--share-gpu" in sys.argv:
    # N ranks on ONE GPU: one hardware queue per process keeps every rank's queue resident,
    # so a collective kernel never spins on a rank whose queue the scheduler left unmapped
    # (parallel/custom_ar.py; profiles/r4_ar_skew_*); read at HIP init, so set before torch
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "1")
    # and the IPC collectives' waiting workgroups must leave CUs free for a late rank's kernels
    os.environ.setdefault("DOCQA_AR_MAX_WG", "32")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    # 256 questions per rank per step: round 3 measured 153 q/s at p50 1.71 s with unique
    # questions (BENCH_r03; the reference-equivalent serial stack: 0.615 q/s, p50 1.62 s,
    # BASELINE.md).  Smaller batches trade throughput for latency: 128 gave ~117 q/s at
    # ~1.16 s p50 in round 1 (profiles/r1_bench_batch_sweep.log, repeated questions)
    ap.add_argument("--batch", type=int, default=256, help="questions per data-parallel rank per step")
    ap.add_argument("--max-new-tokens", type=int, default=128)
    ap.add_argument("--llm", default="llama3-8b")
    ap.add_argument("--embed", default="minilm-l6")
    ap.add_argument("--notes", type=int, default=1000)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--max-context", type=int, default=2048)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--device", default="cuda", help="cuda (MI355X) | cpu (CI rehearsal of the DP path with gloo)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="every rank on cuda:0 (a one-GPU rehearsal of the N-rank DP path; process group "
                         "backend from DOCQA_SHARE_GPU_BACKEND, default gloo); correctness, not speed")
    ap.add_argument("--questions", choices=("unique", "repeat"), default="unique",
                    help="unique: every request a distinct question (default); repeat: the ~470-string "
                         "template grid of rounds 1-2 (cache-hot ceiling)")
    ap.add_argument("--kv-mem-fraction", type=float, default=0.85,
                    help="KV pool = this fraction of the HBM free after the weights (0: max_batch full contexts)")
    ap.add_argument("--template", choices=("cache_friendly", "reference"), default=None,
                    help="QA prompt template (docqa_amd/prompts.py; default: env QA_TEMPLATE, else "
                         "cache_friendly: the headline workload of rounds 2-4, named in the JSON line)")
    ap.add_argument("--check-retrieval", dest="check_retrieval", action="store_true", default=None,
                    help="after the timed region, check every rank's sharded top-k against an unsharded "
                         "flat search over the whole corpus (exit 3 on a mismatch); untimed.  Default: on "
                         "whenever WORLD_SIZE > 1 (the sharded index), off on one GPU")
    ap.add_argument("--no-check-retrieval", dest="check_retrieval", action="store_false")
    a = ap.parse_args()
    os.environ["QA_TEMPLATE"] = a.template or os.environ.get("QA_TEMPLATE", "cache_friendly")

    import torch
    import torch.distributed as dist

    from docqa_amd import ops
    from docqa_amd.engine.llm_engine import SamplingParams
    from docqa_amd.parallel import comm
    from docqa_amd.pipeline.builder import StackConfig, build_stack
    from docqa_amd.text.synthetic import synthetic_questions, synthetic_unique_questions

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print(f"[bench] warning: --gpus {a.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    local_rank = 0 if a.share_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    cuda = a.device == "cuda"
    if cuda:
        torch.cuda.set_device(local_rank)
    backend = None if cuda else "gloo"
    if a.share_gpu:
        backend = os.environ.get("DOCQA_SHARE_GPU_BACKEND", "gloo")
        if backend == "nccl":
            os.environ["LOCAL_RANK"] = "0"    # init_distributed binds the rank to LOCAL_RANK's device
    ps = comm.init_distributed(tp_size=a.tp, backend=backend)
    if cuda:
        assert ops.load_native(), "native HIP kernels not built (python -m docqa_amd.ops.build)"
        # TP > 1: init_distributed already set up the IPC all-reduce (fused residual + RMSNorm,
        # one-/two-shot over all xGMI links) unless DOCQA_CUSTOM_AR=0; RCCL otherwise
    dev = f"cuda:{local_rank}" if cuda else "cpu"

    def sync():
        if cuda:
            torch.cuda.synchronize()

    sc = StackConfig(llm=a.llm, embed=a.embed, n_notes=a.notes, max_batch=a.batch,
                     max_context=a.max_context, k=a.k, use_graphs=(not a.no_graphs) and cuda,
                     kv_mem_fraction=a.kv_mem_fraction or None)
    pipe, info = build_stack(sc, device=dev)
    params = SamplingParams(max_new_tokens=a.max_new_tokens, temperature=0.0, stop_on_eos=False)

    # distinct questions per (step, dp rank); identical within a TP group
    total_steps = a.warmup + a.steps
    gen_q = synthetic_unique_questions if a.questions == "unique" else synthetic_questions
    qs = gen_q(total_steps * ps.dp_size * a.batch, seed=123)

    def batch_for(step: int) -> list[str]:
        base = (step * ps.dp_size + ps.dp_rank) * a.batch
        return qs[base:base + a.batch]

    # Warm-up and timed runs are separate pipelines, so the timed region contains exactly
    # K batches' worth of embed + search + prompt assembly + generation (batch i+1's
    # embed/search run on a side HIP stream and its prompt assembly on a helper thread
    # while batch i generates) and no collective is pending at the barriers.
    for _ in pipe.answer_pipelined([batch_for(w) for w in range(a.warmup)], params):
        pass
    # the cascade decode graph is first needed once prompt prefixes are cached (after the
    # first warm-up batch): capture it here, not inside the timed steps
    pipe.engine.warm_graphs(a.batch)
    sync()
    comm.barrier()
    sync()
    eng = pipe.engine
    s0 = (eng.stats.prefill_s, eng.stats.decode_s, eng.stats.prompt_tokens, eng.stats.cached_tokens)
    a0 = (eng.stats.attn_kv_blocks, eng.stats.attn_batches)
    t0 = time.perf_counter()
    step_times, stages, chunks = [], [], set()
    for ans, st, lat in pipe.answer_pipelined([batch_for(a.warmup + s) for s in range(a.steps)], params):
        step_times.append(lat)   # per-batch answer latency: prepare start -> answers ready
        stages.append(st)
        for x in ans:
            chunks.update(x.chunk_ids)
    sync()
    comm.barrier()
    sync()
    elapsed = time.perf_counter() - t0

    # the driver's multi-GPU runs verify themselves: a wrong cross-shard merge on real xGMI
    # must fail the run, not change the scaling record silently
    do_check = a.check_retrieval if a.check_retrieval is not None else world > 1
    retrieval = check_retrieval(pipe, batch_for(a.warmup), sync) if do_check else None

    t = torch.tensor([elapsed] + step_times, dtype=torch.float64, device=dev)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed_max = float(t[0])
    steps_max = [float(x) for x in t[1:]]
    queries = ps.dp_size * a.batch * a.steps
    qps = queries / elapsed_max
    s1 = (eng.stats.prefill_s, eng.stats.decode_s, eng.stats.prompt_tokens, eng.stats.cached_tokens)
    a1 = (eng.stats.attn_kv_blocks, eng.stats.attn_batches)
    kc = eng.kv.caches[0][0]
    block_bytes = 2 * kc[0].numel() * kc.element_size()       # K + V of one block, one layer
    # workload descriptors over the whole job's timed questions (every DP rank's batches)
    timed_q = [q for s_ in range(a.steps) for d in range(ps.dp_size)
               for q in qs[((a.warmup + s_) * ps.dp_size + d) * a.batch:((a.warmup + s_) * ps.dp_size + d + 1) * a.batch]]
    seen_before = set(qs[:a.warmup * ps.dp_size * a.batch])
    repeats = 0
    for q in timed_q:
        repeats += q in seen_before
        seen_before.add(q)
    if ps.rank == 0:
        st = {k: round(1e3 * statistics.mean(getattr(x, k) for x in stages), 2)
              for k in ("embed_s", "search_s", "prompt_s", "generate_s")}
        out = {
            "metric": "e2e_qa_queries_per_sec",
            "value": round(qps, 3),
            "unit": "queries/s",
            "n_gpus": ps.world_size,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1e3 * elapsed_max / a.steps, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(qps / REF_EQUIV_QPS, 2),
            "dtype": "bf16",
            "data": "synthetic clinical notes + questions, random-init weights",
            "p50_latency_ms": round(1e3 * statistics.median(steps_max), 2),
            "config": {
                "model": f"{a.llm} generator + {a.embed} embedder + flat-L2 kNN (k={a.k})",
                "global_batch": ps.dp_size * a.batch,
                "seq_len": a.max_context,
                "max_new_tokens": a.max_new_tokens,
                "parallelism": f"dp{ps.dp_size}" + (f"xtp{a.tp}" if a.tp > 1 else ""),
                "index_vectors": info.get("index_vectors"),
                "kv_blocks": info.get("kv_blocks"),
            },
            "stage_ms_mean": st,
            "gen_tokens_per_sec": round(ps.dp_size * a.batch * a.max_new_tokens * a.steps / elapsed_max, 1),
            "avg_prompt_tokens": round(eng.stats.prompt_tokens / max(1, (a.warmup + a.steps) * a.batch), 1),
            "engine_ms_per_batch": {"prefill": round(1e3 * (s1[0] - s0[0]) / a.steps, 2),
                                    "decode": round(1e3 * (s1[1] - s0[1]) / a.steps, 2)},
            "prefix_cached_frac": round((s1[3] - s0[3]) / max(1, s1[2] - s0[2]), 3),
            # distinct KV bytes one layer's decode attention must read at a batch's first
            # decode step (cascade prefix once): the HBM floor of that kernel
            "decode_attn_kv_mb_per_layer": round((a1[0] - a0[0]) * block_bytes / max(1, a1[1] - a0[1]) / 1e6, 1),
            "decode_attn_kv_blocks": round((a1[0] - a0[0]) / max(1, a1[1] - a0[1]), 1),
            "kv_block_tokens": eng.block_size,
            "workload": {
                "questions": a.questions,
                "template": os.environ["QA_TEMPLATE"],
                "unique_question_frac": round(len(set(timed_q)) / max(1, len(timed_q)), 4),
                "repeat_of_earlier_frac": round(repeats / max(1, len(timed_q)), 4),
                "distinct_chunks_rank0": len(chunks),
                "context_order": pipe.context_order,
            },
        }
        if retrieval is not None:
            out["retrieval_check"] = retrieval
        if world > 1:
            out["shard_gather"] = getattr(pipe.index, "ipc_status", "process-group gather")
        if cuda:   # the box: CU count and clocks differ between pool machines
            pr = torch.cuda.get_device_properties(local_rank)
            out["device"] = {"name": pr.name, "cus": pr.multi_processor_count,
                             "gcn_arch": getattr(pr, "gcnArchName", "")}
        print(json.dumps(out), flush=True)
    comm.destroy()
    if retrieval is not None and retrieval["bad_rows_max_over_ranks"]:
        sys.exit(3)


def check_retrieval(pipe, questions: list[str], sync) -> dict:
    """The sharded search (IPC gathers + merge, whatever the world size) against ONE exact
    flat L2 index over every record, on the same questions: each row's k distances must
    match, and each returned id's true distance must equal its reported one (duplicated
    KB rows make ids of equal distance interchangeable, so ids are checked by distance).
    Collective: every rank calls it.  Reference: the k=3 retrieval of llm-qa/main.py:101."""
    import torch
    import torch.distributed as dist

    from docqa_amd.index.flat import FlatIndex
    from docqa_amd.pipeline.corpus import embed_records

    k = pipe.k
    dev = pipe.engine.device
    full_x = embed_records(pipe.encoder, pipe.enc_tok, pipe.metadata).float()
    full = FlatIndex(full_x.shape[1], "l2", dev, torch.float32, capacity=max(1024, full_x.shape[0]))
    full.add(full_x)
    q = pipe.embed(questions).float()
    Ds, Is = pipe.index.search(q, k)
    ids = pipe._host_ids(Is)                     # raises on a failed IPC gather
    Df, _ = full.search(q, k)
    sync()
    Ds, Df = Ds.float().cpu(), Df.float().cpu()
    xs = full_x.cpu()
    qc = q.cpu()
    bad = 0
    for r, row in enumerate(ids):
        true = torch.stack([((qc[r] - xs[i]) ** 2).sum() if 0 <= i < xs.shape[0] else torch.tensor(float("inf"))
                            for i in row])
        tol = 1e-3 * (1.0 + Df[r].abs().max())
        if not (torch.allclose(Ds[r], Df[r], atol=tol) and torch.allclose(true, Ds[r], atol=tol)):
            bad += 1
    t = torch.tensor([bad], dtype=torch.int64, device=dev)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return {"rows": len(ids), "k": k, "bad_rows_max_over_ranks": int(t.item())}


if __name__ == "__main__":
    main()
