"""Retrieval-augmented QA: question -> embed -> kNN top-k -> "stuff" prompt -> generate.

Batched and device-resident end to end: a batch of questions is embedded in one packed
varlen encoder forward, searched in one fused distance+top-k launch (or the sharded
all-gather search across GPUs), and all prompts are generated together by the HIP-graph
decode engine.  Per-stage wall times are recorded for the latency breakdown.

Reference parity (llm-qa/main.py:71-122): ``RetrievalQA.from_chain_type(chain_type=
"stuff", k=3, return_source_documents=True)`` -> contexts joined with a blank line into
the prompt's ``{context}``, the user question into ``{question}``; the response carries
``answer`` and the ``source`` metadata of the k retrieved chunks (duplicates allowed).
The reference serves one request at a time; here every stage is batched.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field

import torch

# safety factor of the adaptive pipeline lead (answer_pipelined): preparation cost x this,
# over the decode step time
_LEAD_MARGIN = float(os.environ.get("DOCQA_PIPELINE_LEAD_MARGIN", "1.5"))

from ..utils import tracing
from ..engine.llm_engine import LLMEngine, SamplingParams
from ..prompts import CACHE_FRIENDLY_QA_TEMPLATE, REFERENCE_QA_TEMPLATE, qa_template

# QA prompt: the verbatim reference QA_CHAIN_PROMPT (llm-qa/main.py:71-93) by default, the
# cache-friendly reordering with QA_TEMPLATE=cache_friendly (docqa_amd/prompts.py)
DEFAULT_TEMPLATE = REFERENCE_QA_TEMPLATE


@dataclass
class StageTimes:
    embed_s: float = 0.0
    search_s: float = 0.0
    prompt_s: float = 0.0
    generate_s: float = 0.0

    def total(self) -> float:
        return self.embed_s + self.search_s + self.prompt_s + self.generate_s


@dataclass
class Answer:
    answer: str
    sources: list
    token_ids: list = field(default_factory=list)
    chunk_ids: list = field(default_factory=list)   # index rows retrieved for the prompt


class RAGPipeline:
    def __init__(self, encoder, enc_tokenizer, index, metadata: list[dict], engine: LLMEngine,
                 chat_tokenizer, k: int = 3, template: str | None = None,
                 max_prompt_tokens: int | None = None, context_order: str | None = None):
        template = template if template is not None else qa_template()
        # order of the retrieved chunks inside the prompt: "relevance" (nearest first, as
        # the reference's stuff chain), "shared" (the batch's most-retrieved chunks first,
        # ties by id: prompts retrieving a common chunk then share its KV blocks in the
        # prefix cache) or "trie" (the order whose leading chunks an earlier prompt already
        # used -- this batch or an earlier one, whose KV the prefix cache still holds --
        # else "shared").  Same chunks either way; Answer.sources keep relevance order.
        # Default: trie with the cache-friendly template (the prompt arranged for the prefix
        # cache: 0.72 -> 0.75 -> 0.77 of prompt tokens cached, +5 % then +2.5 % q/s same box,
        # profiles/r4_context_order_ab.log), relevance with the reference's verbatim template
        context_order = context_order or os.environ.get("DOCQA_CONTEXT_ORDER") or (
            "trie" if template == CACHE_FRIENDLY_QA_TEMPLATE else "relevance")
        if context_order not in ("relevance", "shared", "trie"):
            raise ValueError(f"context_order must be relevance, shared or trie, got {context_order!r}")
        self.context_order = context_order
        self._seen: set[tuple[int, ...]] = set()
        self.encoder = encoder
        self.enc_tok = enc_tokenizer
        self.index = index
        self.metadata = metadata
        self.engine = engine
        self.chat_tok = chat_tokenizer
        self.k = k
        self.template = template
        self.max_prompt_tokens = max_prompt_tokens
        self.last_times = StageTimes()
        # token ids of every retrieved chunk, tokenised once: a prompt is then assembled
        # from cached pieces split at paragraph boundaries (the byte-level BPE never merges
        # across a newline pre-token), so only the question is tokenised per request
        self._chunk_ids: dict[int, list[int]] = {}
        self._pieces = None
        if hasattr(chat_tokenizer, "special") and template.count("{context}") == 1 \
                and template.count("{question}") == 1 and template.index("{context}") < template.index("{question}"):
            head, _, rest = template.partition("{context}")
            mid, _, tail = rest.partition("{question}")
            self._pieces = (head, mid, tail)

    def _sync(self):
        if self.engine.device.type == "cuda":
            torch.cuda.synchronize()

    def embed(self, texts: list[str]) -> torch.Tensor:
        return self.encoder.encode(self.enc_tok.encode_batch(texts))

    def _host_ids(self, I: torch.Tensor) -> list[list[int]]:
        """Hits to the host (the batch's one sync on the search stream), then surface a
        failed cross-rank gather of a sharded index (index/sharded.py) as an exception
        instead of serving stale peer rows."""
        ids = I.tolist()
        check = getattr(self.index, "check_gather", None)
        if check is not None:
            check()
        return ids

    def retrieve(self, questions: list[str]):
        """(D, I) of the questions' top-k.  On a sharded index the hits are checked for a
        failed cross-rank gather here (one host sync on the search's ids) so no caller can
        use stale peer rows unchecked."""
        q = self.embed(questions)
        D, I = self.index.search(q, self.k)
        if getattr(self.index, "check_gather", None) is not None:
            self._host_ids(I)
        return D, I

    def _piece_prompt(self, qtext: str, ids: list[int], qids: list[int] | None = None) -> list[int]:
        ct = self.chat_tok
        if not hasattr(self, "_frame"):
            s = ct.special
            head, mid, tail = self._pieces
            self._frame = ([s("<|begin_of_text|>"), s("<|start_header_id|>")] + ct.encode("user")
                           + [s("<|end_header_id|>")] + ct.encode("\n\n" + head),
                           ct.encode("\n\n"), ct.encode(mid),
                           ct.encode(tail) + [s("<|eot_id|>"), s("<|start_header_id|>")] + ct.encode("assistant")
                           + [s("<|end_header_id|>")] + ct.encode("\n\n"))
        pre, sep, mid_ids, post = self._frame
        out = list(pre)
        first = True
        for i in ids:
            if not 0 <= i < len(self.metadata):
                continue
            c = self._chunk_ids.get(i)
            if c is None:
                c = self._chunk_ids[i] = ct.encode(self.metadata[i]["text_content"])
            if not first:
                out += sep
            out += c
            first = False
        return out + mid_ids + (qids if qids is not None else ct.encode(qtext)) + post

    def _ordered(self, I: list[list[int]]) -> list[list[int]]:
        if self.context_order == "relevance":
            return I
        cnt: dict[int, int] = {}
        for ids in I:
            for i in ids:
                cnt[i] = cnt.get(i, 0) + 1
        if self.context_order == "shared":
            return [sorted(ids, key=lambda i: (-cnt[i], i)) for ids in I]
        # "trie": the permutation whose leading chunks an earlier prompt (this batch or an
        # earlier one) already used, longest match first, then batch popularity
        import itertools

        seen = self._seen
        out = []
        for ids in I:
            base = sorted(ids, key=lambda i: (-cnt[i], i))
            best, best_m = base, -1
            if len(ids) <= 4:
                for perm in itertools.permutations(base):
                    m = 0
                    while m < len(perm) and perm[:m + 1] in seen:
                        m += 1
                    if m > best_m:
                        best, best_m = list(perm), m
            for m in range(1, len(best) + 1):
                seen.add(tuple(best[:m]))
            out.append(best)
        if len(seen) > 1_000_000:
            seen.clear()
        return out

    def build_prompts(self, questions: list[str], I: list[list[int]]) -> list[list[int]]:
        I = self._ordered(I)
        if self._pieces is not None and os.environ.get("DOCQA_PROMPT_PIECES", "1") == "1":
            many = getattr(self.chat_tok, "encode_many", None)
            qids = many(questions) if many else [None] * len(questions)
            prompts = [self._piece_prompt(q, ids, qi) for q, ids, qi in zip(questions, I, qids)]
            lim = self.max_prompt_tokens
            if lim:
                prompts = [p if len(p) <= lim else p[: lim // 2] + p[-lim // 2:] for p in prompts]
            return prompts
        texts = []
        for qtext, ids in zip(questions, I):
            ctx = "\n\n".join(self.metadata[i]["text_content"] for i in ids if 0 <= i < len(self.metadata))
            texts.append(self.template.format(context=ctx, question=qtext))
        enc = getattr(self.chat_tok, "encode_batch_chat", None)
        prompts = enc(texts) if enc else [self.chat_tok.chat_prompt(t) for t in texts]
        lim = self.max_prompt_tokens
        if lim:
            prompts = [p if len(p) <= lim else p[: lim // 2] + p[-lim // 2:] for p in prompts]
        return prompts

    @torch.inference_mode()
    def answer_batch(self, questions: list[str], params: SamplingParams | None = None) -> list[Answer]:
        params = params or SamplingParams(stop_on_eos=True)
        t = StageTimes()
        t0 = time.perf_counter()
        with tracing.span("rag.embed", n=len(questions)):
            qemb = self.embed(questions)
            self._sync()
        t1 = time.perf_counter()
        with tracing.span("rag.search", n=len(questions), k=self.k):
            D, I = self.index.search(qemb, self.k)
            I = self._host_ids(I)  # host needs ids to assemble the prompts
        t2 = time.perf_counter()
        with tracing.span("rag.prompt", n=len(questions)):
            prompts = self.build_prompts(questions, I)
        t3 = time.perf_counter()
        with tracing.span("rag.generate", n=len(prompts)):
            outs = self.engine.generate(prompts, params)
        t4 = time.perf_counter()
        t.embed_s, t.search_s, t.prompt_s, t.generate_s = t1 - t0, t2 - t1, t3 - t2, t4 - t3
        self.last_times = t
        res = []
        for ids, toks in zip(I, outs):
            srcs = [self.metadata[i].get("source") for i in ids if 0 <= i < len(self.metadata)]
            res.append(Answer(answer=self.chat_tok.decode(toks), sources=srcs, token_ids=toks,
                              chunk_ids=list(ids)))
        return res

    def answer(self, question: str, params: SamplingParams | None = None) -> Answer:
        return self.answer_batch([question], params)[0]

    # ------------------------------------------------------------------ pipelined
    @torch.inference_mode()
    def _prepare(self, questions: list[str], stream, gate, params=None):
        """embed + kNN on a side HIP stream (held back by ``gate`` until the running
        generation is ``lead_steps`` from its end), then host-side prompt assembly and
        (``params`` given) the batch's KV-block reservation."""
        t0 = time.perf_counter()
        evs = None
        sp = tracing.span("rag.prepare", n=len(questions))
        sp.__enter__()
        if stream is not None:
            with torch.cuda.stream(stream):
                if gate is not None:
                    stream.wait_event(gate)
                # GPU-clock stage times: embed = [e0, e1), kNN search = [e1, e2)
                evs = tuple(torch.cuda.Event(enable_timing=True) for _ in range(3))
                evs[0].record(stream)
                qemb = self.embed(questions)
                evs[1].record(stream)
                _, I = self.index.search(qemb, self.k)
                evs[2].record(stream)
                I = self._host_ids(I)       # waits for this side stream only
            host = None
        else:
            qemb = self.embed(questions)
            tm = time.perf_counter()
            _, I = self.index.search(qemb, self.k)
            I = self._host_ids(I)
            host = (tm - t0, time.perf_counter() - tm)
        t1 = time.perf_counter()
        with tracing.span("rag.prompts", n=len(questions)):
            prompts = self.build_prompts(questions, I)
        reserved = None
        if params is not None and len(prompts) <= self.engine.max_batch:
            try:
                reserved = self.engine.reserve(prompts, params)
            except MemoryError:
                # the batches still in flight hold the pool: the main loop collects them
                # first and reserves this batch itself (reserved=None)
                reserved = None
        sp.__exit__(None, None, None)
        return questions, I, prompts, reserved, (evs, host), t0, t1, time.perf_counter()

    @torch.inference_mode()
    def answer_pipelined(self, batches: list[list[str]], params: SamplingParams | None = None,
                         lead_steps: int | None = None):
        """Yield (answers, StageTimes, latency_s) per batch.  Batch i+1's embedding and
        kNN search run on a side HIP stream and its prompt assembly + KV reservation on a
        helper thread, released when batch i's decode is ``lead_steps`` steps from its
        end, so they overlap the tail of batch i's generation; batch i+1 is then launched
        (prefill + decode graphs queued behind batch i) before batch i is collected and
        detokenised on a second helper thread, so the GPU never waits on host work between
        batches.  Latency is measured on the GPU clock from the moment batch i+1's
        embedding may start to its answers being ready."""
        import concurrent.futures as cf

        params = params or SamplingParams(stop_on_eos=True)
        # embed + kNN (side stream) + prompt assembly + KV reservation of batch i+1 should
        # finish before batch i's last decode step, so batch i+1's prefill is queued right
        # behind it (launch-before-collect below); an earlier start only adds latency
        # (measured: lead 4 / 8 / 16 steps -> 205.1 / 204.8 / 204.4 q/s, p50 1264 / 1301 /
        # 1370 ms; profiles/r2_ab_pipeline_lead.log).  Adaptive (no argument, no env): after
        # the first batch the lead is the measured preparation time over the measured decode
        # step time, x1.5 -- 1 step at batch 1 (1.5 ms of preparation vs 3.6 ms steps; a
        # fixed 4 put 11 ms of waiting into every answer's latency), 4 at batch 256
        env_lead = os.environ.get("DOCQA_PIPELINE_LEAD")
        # data-parallel ranks keep the fixed lead: their batch preparation meets in the
        # sharded index's all-gather, so every rank must release it at the same step
        dp = torch.distributed.is_available() and torch.distributed.is_initialized() and \
            torch.distributed.get_world_size() > 1
        adaptive = lead_steps is None and env_lead is None and not dp
        lead = [lead_steps if lead_steps is not None else int(env_lead or 4)]
        est = {"prep": None, "step": None}

        def adapt():
            if adaptive and est["prep"] is not None and est["step"]:
                lead[0] = max(1, min(16, math.ceil(_LEAD_MARGIN * est["prep"] / est["step"])))
        eng = self.engine
        cuda = eng.device.type == "cuda"
        stream = torch.cuda.Stream() if cuda else None
        pending = None   # (Launched, questions, I, stage timers, t0, t1, t2, t3) of the batch in flight

        def stage_times(tm, t0, t1, t2, gen_s):
            evs, host = tm
            if evs is not None:
                emb, srch = evs[0].elapsed_time(evs[1]) / 1e3, evs[1].elapsed_time(evs[2]) / 1e3
            else:
                emb, srch = host if host is not None else (t1 - t0, 0.0)
            return StageTimes(embed_s=emb, search_s=srch, prompt_s=t2 - t1, generate_s=gen_s)

        def finish(p):
            h, questions, I, tm, t0, t1, t2, t3 = p
            outs = eng.collect(h)
            t4 = time.perf_counter()
            if cuda:
                latency = tm[0][0].elapsed_time(h.done_event) / 1e3
                gen_s = h.start_event.elapsed_time(h.done_event) / 1e3
            else:
                latency, gen_s = t4 - t0, t4 - t3
            est["step"] = gen_s / max(1, params.max_new_tokens)
            adapt()
            st = stage_times(tm, t0, t1, t2, gen_s)
            self.last_times = st
            with tracing.span("rag.detokenise", n=len(outs)):
                res = [Answer(answer=self.chat_tok.decode(toks),
                              sources=[self.metadata[j].get("source") for j in ids if 0 <= j < len(self.metadata)],
                              token_ids=toks, chunk_ids=list(ids)) for ids, toks in zip(I, outs)]
            return res, st, latency

        # batch i-1 is collected and detokenised on a helper thread as soon as batch i's
        # decode starts being enqueued (its prefill is queued by then): enqueueing the
        # decode graphs blocks the host on the stream's queue depth until about the end of
        # the batch, so collecting after launch() returned left the GPU idle meanwhile
        with cf.ThreadPoolExecutor(1, thread_name_prefix="rag-prep") as ex, \
                cf.ThreadPoolExecutor(1, thread_name_prefix="rag-collect") as col:
            fut = ex.submit(self._prepare, batches[0], stream, None, params) if batches else None
            fin = None
            try:
                for i in range(len(batches)):
                    questions, I, prompts, reserved, tm, t0, t1, t2 = fut.result()
                    fut = None
                    # preparation cost, not the wait for the gate: GPU embed + search time (side
                    # stream events, complete once the host has the hits) + host prompt assembly
                    evs = tm[0] if tm is not None else None
                    est["prep"] = ((evs[0].elapsed_time(evs[2]) / 1e3 + (t2 - t1)) if evs is not None
                                   else t2 - t0)
                    adapt()
                    nxt = batches[i + 1] if i + 1 < len(batches) else None

                    def on_step(step, total, nxt=nxt):
                        nonlocal fut, fin, pending
                        if pending is not None and fin is None:
                            p, pending = pending, None
                            fin = col.submit(finish, p)
                        if nxt is not None and fut is None and step >= max(1, total - lead[0]):
                            gate = None
                            if cuda:
                                gate = torch.cuda.Event()
                                gate.record()
                            fut = ex.submit(self._prepare, nxt, stream, gate, params)

                    if reserved is None and pending is not None and len(prompts) <= eng.max_batch:
                        # no KV reservation (pool held by the batch in flight): collect that
                        # batch first so launch() can reserve this one
                        p, pending = pending, None
                        yield finish(p)
                    t3 = time.perf_counter()
                    if len(prompts) <= eng.max_batch:
                        h = eng.launch(prompts, params, on_step=on_step, reserved=reserved)
                    else:   # larger than one engine batch: plain blocking generation
                        h = None
                        outs = eng.generate(prompts, params, on_step=on_step)
                    if nxt is not None and fut is None:   # single-step generations
                        fut = ex.submit(self._prepare, nxt, stream, None, params)
                    if pending is not None:   # no decode step enqueued: collect batch i-1 now
                        p, pending = pending, None
                        fin = col.submit(finish, p)
                    if fin is not None:
                        f, fin = fin, None
                        yield f.result()
                    if h is not None:
                        pending = (h, questions, I, tm, t0, t1, t2, t3)
                    else:
                        t4 = time.perf_counter()
                        st = stage_times(tm, t0, t1, t2, t4 - t3)
                        self.last_times = st
                        yield ([Answer(answer=self.chat_tok.decode(toks),
                                       sources=[self.metadata[j].get("source") for j in ids
                                                if 0 <= j < len(self.metadata)], token_ids=toks,
                                       chunk_ids=list(ids))
                                for ids, toks in zip(I, outs)], st, t4 - t0)
                if pending is not None:
                    p, pending = pending, None
                    yield finish(p)
            finally:
                if fin is not None:
                    try:
                        fin.result()
                    except Exception:
                        pass
                if pending is not None:   # abandoned generator: wait, free the blocks
                    eng.collect(pending[0])
                if fut is not None:
                    try:
                        r = fut.result()[3]
                        if r is not None:
                            eng.release(r)
                    except Exception:
                        pass


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
