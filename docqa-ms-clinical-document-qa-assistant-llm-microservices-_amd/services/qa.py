"""llm-qa service (FastAPI, port 8001; 8004 in the synthese deployment).

Contract (llm-qa/main.py:108-126 and synthese-comparative/core/llm_client.py:42-54):
  POST /ask/                {"question"} -> {"answer", "sources": [source x k]}
                            503 {"detail": "Index non chargé."} when no index is loaded
  POST /api/llm/summarize   {"prompt"}   -> {"summary"}   (expected by synthese, missing
                            in the reference; served here)
  GET  /health              {"status": "ok", "service": "llm-qa"}
  GET  /metrics             Prometheus text (requests, batch sizes, stage latencies)
  POST /api/chat, /api/generate, GET /api/tags, /api/version
                            the Ollama wire API the reference's ChatOllama posts to
                            (services/ollama_api.py), served from this engine

Serving model: the reference answers one blocking request at a time per process
(llm-qa/main.py:111-117).  Here (``DOCQA_SERVING=continuous``, default) a prep thread
takes every request that arrived, embeds and searches them as one batch on a side HIP
stream and hands their prompts to the continuous-batching engine (engine/scheduler.py),
whose scheduler thread admits them into the running decode batch at the next step; they
leave it when they finish -- no request waits for another batch to drain, and question
embedding overlaps the decode steps instead of pausing them.
``DOCQA_SERVING=batch`` keeps the static dynamic batcher: drain the queue every
``BATCH_WINDOW_MS`` (or at ``MAX_BATCH``) and run the batch from prefill to last token.
"""
from __future__ import annotations

import asyncio
import concurrent.futures as cf
import os
import queue
import threading
import time

from fastapi import FastAPI
from fastapi.responses import JSONResponse, PlainTextResponse

from ..config import Settings
from ..engine.llm_engine import SamplingParams
from ..schemas import AskResponse, Query, SummarizeRequest, SummarizeResponse
from ..utils import tracing
from ..utils.metrics import Metrics


class DynamicBatcher:
    def __init__(self, pipeline, settings: Settings, metrics: Metrics):
        self.pipe = pipeline
        self.st = settings
        self.metrics = metrics
        self.q: queue.Queue = queue.Queue()
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._loop, name="qa-batcher", daemon=True)
        self._t.start()

    def submit(self, kind: str, payload: str) -> cf.Future:
        f: cf.Future = cf.Future()
        self.q.put((kind, payload, f, time.perf_counter()))
        return f

    def _params(self) -> SamplingParams:
        return SamplingParams(max_new_tokens=self.st.max_new_tokens, temperature=self.st.temperature,
                              stop_on_eos=self.st.stop_on_eos)

    def _loop(self) -> None:
        while not self._stop.is_set():
            try:
                first = self.q.get(timeout=0.1)
            except queue.Empty:
                continue
            batch = [first]
            deadline = time.perf_counter() + self.st.batch_window_ms / 1e3
            while len(batch) < self.st.max_batch:
                rem = deadline - time.perf_counter()
                if rem <= 0:
                    break
                try:
                    batch.append(self.q.get(timeout=rem))
                except queue.Empty:
                    break
            self._run(batch)

    def _run(self, batch) -> None:
        asks = [b for b in batch if b[0] == "ask"]
        sums = [b for b in batch if b[0] == "summarize"]
        try:
            if asks:
                res = self.pipe.answer_batch([b[1] for b in asks], self._params())
                for (_, _, f, t0), r in zip(asks, res):
                    self.metrics.observe("ask_latency_s", time.perf_counter() - t0)
                    f.set_result({"answer": r.answer, "sources": r.sources})
                self.metrics.observe("ask_batch_size", len(asks))
                for k, v in vars(self.pipe.last_times).items():
                    self.metrics.observe(f"stage_{k}", v)
            gens = [b for b in batch if b[0] == "gen"]
            # Ollama-API requests: raw prompt ids with their own sampling options, one engine
            # batch per distinct option set (no token streaming on this path)
            groups: dict = {}
            for b in gens:
                p = b[1]["params"]
                groups.setdefault((p.max_new_tokens, p.temperature, p.top_k, p.top_p, p.stop_on_eos, p.seed),
                                  []).append(b)
            for grp in groups.values():
                outs = self.pipe.engine.generate([b[1]["ids"] for b in grp], grp[0][1]["params"])
                for (_, _, f, t0), o in zip(grp, outs):
                    self.metrics.observe("generate_latency_s", time.perf_counter() - t0)
                    f.set_result({"ids": list(o)})
            if sums:
                prompts = [self.pipe.chat_tok.chat_prompt(b[1]) for b in sums]
                lim = self.pipe.max_prompt_tokens
                if lim:
                    prompts = [p if len(p) <= lim else p[: lim // 2] + p[-lim // 2:] for p in prompts]
                outs = self.pipe.engine.generate(prompts, self._params())
                for (_, _, f, t0), o in zip(sums, outs):
                    self.metrics.observe("summarize_latency_s", time.perf_counter() - t0)
                    f.set_result({"summary": self.pipe.chat_tok.decode(o)})
        except Exception as e:  # noqa: BLE001 - fail every waiter of the batch
            for b in batch:
                if not b[2].done():
                    b[2].set_exception(e)

    def stop(self) -> None:
        self._stop.set()
        self._t.join(timeout=60)


def _maybe_exit_on_device_error(e: Exception) -> None:
    """A HIP error is sticky: the process's GPU context cannot serve again.  Under the
    supervisor (DOCQA_EXIT_ON_DEVICE_ERROR=1) exit so it restarts this service; otherwise
    keep serving the error to clients (every later request fails fast)."""
    import os

    msg = f"{type(e).__name__}: {e}"
    if os.environ.get("DOCQA_EXIT_ON_DEVICE_ERROR") == "1" and ("HIP error" in msg or "AcceleratorError" in msg):
        import logging

        logging.getLogger("llm-qa").critical("device error, exiting for a supervised restart: %s", msg)
        os._exit(70)


class ContinuousBatcher:
    """Two threads: the prep thread takes every request that arrived, embeds and searches
    them as one batch on a side HIP stream and submits their prompts to the
    continuous-batching engine; the scheduler thread only runs engine steps (admission
    prefills + decode).  Question embedding therefore never stalls the decode loop -- with
    the embed inline, every arrival burst under load cost the running batch a step."""

    def __init__(self, pipeline, settings: Settings, metrics: Metrics, lockstep=None):
        from ..engine.scheduler import ContinuousEngine

        self.pipe = pipeline
        self.st = settings
        self.metrics = metrics
        # lockstep: this process leads a tensor-parallel group whose other ranks mirror
        # every engine step (engine/scheduler.py Lockstep; services/launch.py --tp)
        self.engine = ContinuousEngine(pipeline.engine, max_running=settings.max_batch, lockstep=lockstep)
        if os.environ.get("DOCQA_WARM_BUCKETS", "1") == "1":
            # every decode bucket captured before the first request (the TP followers do
            # the same before following, services/launch.py)
            self.engine.warmup()
        self.q: queue.Queue = queue.Queue()
        self._prep_window_s = float(os.environ.get("DOCQA_PREP_WINDOW_MS", "0")) / 1e3
        self._stop = threading.Event()
        self._prep = threading.Thread(target=self._prep_loop, name="qa-prep", daemon=True)
        self._t = threading.Thread(target=self._loop, name="qa-scheduler", daemon=True)
        self._prep.start()
        self._t.start()

    def submit(self, kind: str, payload: str) -> cf.Future:
        f: cf.Future = cf.Future()
        self.q.put((kind, payload, f, time.perf_counter()))
        return f

    def _params(self) -> SamplingParams:
        return SamplingParams(max_new_tokens=self.st.max_new_tokens, temperature=self.st.temperature,
                              stop_on_eos=self.st.stop_on_eos)

    def _drain(self) -> list:
        """Everything queued now; while the engine is busy, also what arrives within
        DOCQA_PREP_WINDOW_MS of the first item (default 0: off).  Under load every arrival
        gets its own embed + search launches on the side stream (prep batches of one request
        at 320 q/s, ~7 % of the kernel time); a 4 / 8 ms window groups 3-4 requests per prep
        batch but measured no faster (steady 130.4 / 129.2 vs 129.6 q/s at Poisson 320,
        profiles/r3c_serve_ab_prep.log): the side-stream work overlaps the decode steps."""
        items = []
        try:
            items.append(self.q.get(timeout=0.1))
        except queue.Empty:
            return items
        deadline = time.perf_counter() + (self._prep_window_s if self.engine.has_work() else 0.0)
        while len(items) < self.st.max_batch:
            rem = deadline - time.perf_counter()
            try:
                items.append(self.q.get(timeout=rem) if rem > 0 else self.q.get_nowait())
            except queue.Empty:
                return items
        return items

    def _prep_loop(self) -> None:
        import torch

        cuda = self.pipe.engine.device.type == "cuda"
        side = torch.cuda.Stream() if cuda else None
        while not self._stop.is_set():
            items = self._drain()
            if not items:
                continue
            try:
                with torch.inference_mode(), (torch.cuda.stream(side) if cuda else _nullctx()):
                    self._admit(items)
            except Exception as e:  # noqa: BLE001
                for it in items:
                    if not it[2].done():
                        it[2].set_exception(e)

    def _loop(self) -> None:
        from ..parallel.health import Watchdog

        # DOCQA_WATCHDOG_S=<s>: exit (for a supervised restart) when a step hangs that long
        wd = Watchdog.from_env()
        eng = self.engine
        while not self._stop.is_set():
            if not eng.has_work():
                if wd:
                    wd.idle()
                with eng._cv:
                    if not eng.has_work():
                        eng._cv.wait(timeout=0.05)
                if not eng.has_work():
                    eng.heartbeat()          # TP followers: keep their receive alive
                continue
            if wd:
                wd.busy()
            try:
                eng.step()
            except Exception as e:  # noqa: BLE001
                import logging

                logging.getLogger("llm-qa").error("engine step failed: %s: %s", type(e).__name__, e)
                try:
                    eng._fail_all(e)      # fails every running request's future first
                except Exception as e2:  # noqa: BLE001 - the loop must survive to fail later requests
                    logging.getLogger("llm-qa").error("engine reset failed: %s: %s", type(e2).__name__, e2)
                _maybe_exit_on_device_error(e)
            m = self.metrics
            m.set("engine_steps", eng.steps)
            m.set("engine_preemptions", eng.preempted)
            m.set("engine_kv_admission_blocked", eng.kv_blocked)
            m.set("engine_generated_tokens", eng.generated)
            m.set("engine_completed", eng.completed)
            m.set("engine_completed_short", eng.completed_short)
            if wd:
                wd.beat()
        if wd:
            wd.stop()

    def _admit(self, items) -> None:
        pipe, params = self.pipe, self._params()
        asks = [it for it in items if it[0] == "ask"]
        sums = [it for it in items if it[0] == "summarize"]
        if asks:
            tp0 = time.perf_counter()
            qs = [it[1] for it in asks]
            qemb = pipe.embed(qs)
            _, I = pipe.index.search(qemb, pipe.k)
            I = pipe._host_ids(I)
            prompts = pipe.build_prompts(qs, I)
            te = time.perf_counter()
            m = self.metrics
            m.observe("ask_batch_size", len(asks))
            m.observe("ask_prep_batch_s", te - tp0)          # embed + search + prompt assembly
            for (_, _, f, t0), ids, p in zip(asks, I, prompts):
                m.observe("ask_queue_s", tp0 - t0)            # arrival -> its prep batch starts
                srcs = [pipe.metadata[j].get("source") for j in ids if 0 <= j < len(pipe.metadata)]

                def done(ef, f=f, t0=t0, srcs=srcs):
                    if ef.exception() is not None:
                        f.set_exception(ef.exception())
                        return
                    now = time.perf_counter()
                    m.observe("ask_latency_s", now - t0)
                    m.observe("ask_engine_s", now - te)      # engine admission + prefill + decode
                    f.set_result({"answer": pipe.chat_tok.decode(ef.result()), "sources": srcs})

                self.engine.submit(p, params).add_done_callback(done)
        for _, g, f, t0 in (it for it in items if it[0] == "gen"):
            # Ollama-API requests (services/ollama_api.py): prompt ids + per-request sampling,
            # tokens streamed through on_token as the scheduler emits them

            def gdone(ef, f=f, t0=t0):
                if ef.exception() is not None:
                    f.set_exception(ef.exception())
                    return
                self.metrics.observe("generate_latency_s", time.perf_counter() - t0)
                f.set_result({"ids": list(ef.result())})

            self.engine.submit(g["ids"], g["params"], g.get("on_token")).add_done_callback(gdone)
        for _, text, f, t0 in sums:
            p = pipe.chat_tok.chat_prompt(text)
            lim = pipe.max_prompt_tokens
            if lim and len(p) > lim:
                p = p[: lim // 2] + p[-lim // 2:]

            def sdone(ef, f=f, t0=t0):
                if ef.exception() is not None:
                    f.set_exception(ef.exception())
                    return
                self.metrics.observe("summarize_latency_s", time.perf_counter() - t0)
                f.set_result({"summary": pipe.chat_tok.decode(ef.result())})

            self.engine.submit(p, params).add_done_callback(sdone)

    def stop(self) -> None:
        self._stop.set()
        self._prep.join(timeout=60)
        self._t.join(timeout=60)
        self.engine.stop_followers()


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class ReplicaRouter:
    """Front-end over data-parallel llm-qa replicas (services/launch.py --gpus N): requests
    go round-robin to this process's own batcher or to another replica's HTTP endpoint,
    with the fewest requests in flight winning ties."""

    def __init__(self, local, urls: list[str], timeout_s: float = 600.0):
        import httpx

        self.local = local
        self.targets = [None] + list(urls)        # None: this process
        self.inflight = [0] * len(self.targets)
        self._rr = 0
        self._lock = threading.Lock()
        self.client = httpx.AsyncClient(timeout=timeout_s)

    def _pick(self) -> int:
        with self._lock:
            n = len(self.targets)
            order = [(self._rr + i) % n for i in range(n)]
            i = min(order, key=lambda k: self.inflight[k])
            self._rr = (i + 1) % n
            self.inflight[i] += 1
            return i

    async def call(self, kind: str, path: str, payload: dict, key: str):
        i = self._pick()
        try:
            if self.targets[i] is None:
                return await asyncio.wrap_future(self.local.submit(kind, payload[key]))
            r = await self.client.post(self.targets[i] + path, json=payload)
            return JSONResponse(status_code=r.status_code, content=r.json())
        finally:
            with self._lock:
                self.inflight[i] -= 1


def create_app(pipeline=None, settings: Settings | None = None, lockstep=None,
               replicas: list[str] | None = None) -> FastAPI:
    """``lockstep``: this process leads a TP group (continuous serving only);
    ``replicas``: base URLs of the other data-parallel llm-qa replicas to balance over."""
    st = settings or Settings()
    metrics = Metrics("llm_qa")
    app = FastAPI(title="Health LLM Assistant (MI355X)")
    app.state.pipeline = pipeline
    batcher_cls = ContinuousBatcher if st.serving_mode == "continuous" else DynamicBatcher
    if lockstep is not None and batcher_cls is not ContinuousBatcher:
        raise ValueError("tensor-parallel serving needs DOCQA_SERVING=continuous")
    kw = {"lockstep": lockstep} if lockstep is not None else {}
    app.state.batcher = batcher_cls(pipeline, st, metrics, **kw) if pipeline is not None else None
    router = ReplicaRouter(app.state.batcher, replicas) if replicas and app.state.batcher is not None else None
    app.state.router = router

    def ready() -> bool:
        p = app.state.pipeline
        return p is not None and p.index is not None and p.index.ntotal > 0

    @app.post("/ask/", response_model=AskResponse)
    async def ask_question(query: Query):
        if not ready():
            return JSONResponse(status_code=503, content={"detail": "Index non chargé."})
        metrics.inc("ask_requests")
        if router is not None:
            return await router.call("ask", "/ask/", {"question": query.question}, "question")
        fut = app.state.batcher.submit("ask", query.question)
        return await asyncio.wrap_future(fut)

    @app.post("/api/llm/summarize", response_model=SummarizeResponse)
    async def summarize(req: SummarizeRequest):
        if app.state.batcher is None:
            return JSONResponse(status_code=503, content={"detail": "LLM non chargé."})
        metrics.inc("summarize_requests")
        if router is not None:
            return await router.call("summarize", "/api/llm/summarize", {"prompt": req.prompt}, "prompt")
        fut = app.state.batcher.submit("summarize", req.prompt)
        return await asyncio.wrap_future(fut)

    # the Ollama wire API the reference's llm-qa calls (ChatOllama, llm-qa/main.py:66-69,117)
    from . import ollama_api

    ollama_api.register(app, st, metrics)

    @app.get("/health")
    def health():
        return {"status": "ok", "service": "llm-qa"}

    @app.get("/metrics")
    def prom():
        return PlainTextResponse(metrics.render())

    @app.get("/debug/trace")
    def trace_dump():
        """Chrome / Perfetto trace-event JSON of the recorded spans (DOCQA_TRACE=1)."""
        return tracing.chrome_trace()

    @app.get("/debug/trace/summary")
    def trace_summary():
        return {"enabled": tracing.enabled(), "spans": tracing.summary()}

    return app
