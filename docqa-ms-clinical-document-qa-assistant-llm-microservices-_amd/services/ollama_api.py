"""Ollama-compatible generation API on the llm-qa service.

The reference's llm-qa does not generate itself: ``ChatOllama(model="mistral",
temperature=0)`` (llm-qa/main.py:66-69) posts every prompt to an external Ollama server
at ``OLLAMA_BASE_URL`` (``/api/chat``, llm-qa/main.py:117; SURVEY §2.4 message-site
table).  Serving the same wire API from this service's engine makes it a drop-in for that
external dependency: a LangChain ``ChatOllama`` / ``ollama`` client pointed at this
service's URL gets its completions from the MI355X engine (continuous batching with every
other request in flight) instead of a llama.cpp process.

  POST /api/chat      {"model", "messages": [{"role", "content"}], "stream" (default true),
                       "options": {"temperature", "num_predict", "top_k", "top_p", "seed"}}
                      -> {"model", "created_at", "message": {"role": "assistant", "content"},
                          "done": true, "done_reason": "stop" | "length", "total_duration",
                          "load_duration", "prompt_eval_count", "prompt_eval_duration",
                          "eval_count", "eval_duration"}
                      stream: application/x-ndjson, one line per text piece
                      ({"message": {..., "content": piece}, "done": false}) then the final
                      line above with an empty content
  POST /api/generate  {"model", "prompt", "system", "raw", "stream", "options"} -> the same
                      with "response" instead of "message"
  GET  /api/tags      the one model this process serves; GET /api/version

Deviations, by design: one model per process (the request's "model" is echoed, not used to
pick weights); "temperature" defaults to the service's TEMPERATURE (0, the reference's
setting) rather than Ollama's 0.8; "format", "keep_alive", "images" and "tools" are ignored.
Durations are nanoseconds like Ollama's.  Streaming is token by token on the continuous
scheduler (DOCQA_SERVING=continuous, the default); the static batcher returns the whole
completion as one piece.
"""
from __future__ import annotations

import asyncio
import json
import time
from datetime import datetime, timezone

from fastapi import FastAPI
from fastapi.responses import JSONResponse, StreamingResponse
from pydantic import BaseModel

from ..engine.llm_engine import SamplingParams

_DONE = object()


class OllamaMessage(BaseModel):
    role: str = "user"
    content: str = ""


class OllamaChatRequest(BaseModel):
    model: str = ""
    messages: list[OllamaMessage] = []
    stream: bool = True
    options: dict | None = None


class OllamaGenerateRequest(BaseModel):
    model: str = ""
    prompt: str = ""
    system: str | None = None
    raw: bool = False
    stream: bool = True
    options: dict | None = None


def _now() -> str:
    return datetime.now(timezone.utc).isoformat().replace("+00:00", "Z")


def sampling_from_options(options: dict | None, settings, max_context: int, prompt_len: int) -> SamplingParams:
    """Ollama ``options`` -> SamplingParams: num_predict (-1 / -2: up to the context) caps
    the new tokens, temperature 0 is greedy."""
    o = options or {}
    n = int(o.get("num_predict", settings.max_new_tokens))
    room = max(1, max_context - prompt_len)
    n = room if n < 0 else max(1, min(n, room))
    return SamplingParams(max_new_tokens=n, temperature=float(o.get("temperature", settings.temperature)),
                          top_k=int(o.get("top_k", 0) or 0), top_p=float(o.get("top_p", 1.0) or 1.0),
                          stop_on_eos=True, seed=int(o.get("seed", 0) or 0))


def register(app: FastAPI, settings, metrics) -> None:
    """Add the Ollama routes to the llm-qa app (``app.state.pipeline`` / ``app.state.batcher``)."""

    def _prompt_ids(pipe, ids: list[int]) -> list[int]:
        lim = pipe.max_prompt_tokens
        return ids if not lim or len(ids) <= lim else ids[: lim // 2] + ids[-(lim // 2):]

    async def _run(kind: str, model: str, ids: list[int], options: dict | None, stream: bool):
        pipe, batcher = app.state.pipeline, app.state.batcher
        if pipe is None or batcher is None:
            return JSONResponse(status_code=503, content={"error": "model not loaded"})
        tok = pipe.chat_tok
        ids = _prompt_ids(pipe, ids)
        params = sampling_from_options(options, settings, pipe.engine.max_context, len(ids))
        metrics.inc(f"ollama_{kind}_requests")
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        t0 = time.perf_counter()
        first = [0.0]

        def on_token(_rid, t):
            if not first[0]:
                first[0] = time.perf_counter()
            loop.call_soon_threadsafe(q.put_nowait, t)

        fut = batcher.submit("gen", {"ids": ids, "params": params, "on_token": on_token if stream else None})
        fut.add_done_callback(lambda f: loop.call_soon_threadsafe(q.put_nowait, _DONE))

        def body(text: str) -> dict:
            if kind == "chat":
                return {"message": {"role": "assistant", "content": text}}
            return {"response": text}

        def final(out: list[int], text: str) -> dict:
            t1 = time.perf_counter()
            tf = first[0] or t1
            eos = bool(out) and out[-1] == pipe.engine.model.cfg.eos_token_id
            d = {"model": model or settings.llm_model, "created_at": _now(), **body(text), "done": True,
                 "done_reason": "stop" if eos else "length", "total_duration": int((t1 - t0) * 1e9),
                 "load_duration": 0, "prompt_eval_count": len(ids), "prompt_eval_duration": int((tf - t0) * 1e9),
                 "eval_count": len(out), "eval_duration": int((t1 - tf) * 1e9)}
            if kind == "generate":
                d["context"] = []
            return d

        if not stream:
            res = await asyncio.wrap_future(fut)
            return JSONResponse(final(res["ids"], tok.decode(res["ids"])))

        async def lines():
            got: list[int] = []
            sent = ""
            while True:
                item = await q.get()
                if item is _DONE:
                    break
                got.append(item)
                text = tok.decode(got)
                if text.endswith("\ufffd"):     # an incomplete UTF-8 sequence: wait for its bytes
                    continue
                piece, sent = text[len(sent):], text
                if piece:
                    yield json.dumps({"model": model or settings.llm_model, "created_at": _now(), **body(piece),
                                      "done": False}) + "\n"
            try:
                out = fut.result()["ids"]
            except Exception as e:  # noqa: BLE001 - the stream is already open: report in-band
                yield json.dumps({"error": f"{type(e).__name__}: {e}"}) + "\n"
                return
            text = tok.decode(out)
            rest = text[len(sent):] if text.startswith(sent) else text
            if rest:     # the static batcher (no per-token callback) or a held-back tail
                yield json.dumps({"model": model or settings.llm_model, "created_at": _now(), **body(rest),
                                  "done": False}) + "\n"
            yield json.dumps(final(out, "")) + "\n"

        return StreamingResponse(lines(), media_type="application/x-ndjson")

    @app.post("/api/chat")
    async def ollama_chat(req: OllamaChatRequest):
        pipe = app.state.pipeline
        if pipe is None:
            return JSONResponse(status_code=503, content={"error": "model not loaded"})
        ids = pipe.chat_tok.chat_messages([m.model_dump() for m in req.messages])
        return await _run("chat", req.model, ids, req.options, req.stream)

    @app.post("/api/generate")
    async def ollama_generate(req: OllamaGenerateRequest):
        pipe = app.state.pipeline
        if pipe is None:
            return JSONResponse(status_code=503, content={"error": "model not loaded"})
        tok = pipe.chat_tok
        if req.raw:
            ids = tok.encode(req.prompt)
        else:
            ids = tok.chat_prompt(req.prompt, system=req.system)
        return await _run("generate", req.model, ids, req.options, req.stream)

    @app.get("/api/tags")
    def ollama_tags():
        pipe = app.state.pipeline
        models = []
        if pipe is not None:
            m = pipe.engine.model
            models.append({"name": settings.llm_model, "model": settings.llm_model, "modified_at": _now(),
                           "size": int(m.weight_bytes()), "digest": "",
                           "details": {"format": "safetensors", "family": "llama", "families": ["llama"],
                                       "parameter_size": f"{m.cfg.num_params() / 1e9:.1f}B",
                                       "quantization_level": "BF16"}})
        return {"models": models}

    @app.get("/api/version")
    def ollama_version():
        return {"version": "0.0.0-docqa-mi355x"}
