"""Online serving benchmark for llm-qa: open-loop Poisson arrivals of clinical questions.

Two entry points:

* ``--entry launch`` (default) -- the deployed service: this script starts
  ``python -m docqa_amd.services.launch --services indexer,qa`` (the same launcher an
  operator runs; ``--gpus N --tp T`` for data/tensor-parallel replicas under torchrun) in
  its own process group, waits until /ask/ answers, and fires the arrivals at
  ``POST /ask/`` over HTTP (httpx).  Latency is arrival -> HTTP response, so it includes
  the FastAPI/uvicorn front end, the batcher, RAG retrieval and generation.  This
  process never touches the GPU.
* ``--entry inproc`` -- the same pipeline in this process, scheduler A/B without HTTP:
  the continuous-batching scheduler (engine/scheduler.py) against the static dynamic
  batcher (``--modes continuous,batch``).

Reports completed queries/s and latency percentiles.  Synthetic questions (unique by
default, ``--questions repeat`` for the 14-template set), random-init weights.  One JSON
line per mode.  Reference parity: the reference has no serving benchmark;
its llm-qa /ask/ (llm-qa/main.py) is the endpoint under load.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import signal
import statistics
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _arrivals(n: int, rate: float, seed: int = 0) -> list[float]:
    rng = random.Random(seed)
    t, out = 0.0, []
    for _ in range(n):
        t += rng.expovariate(rate)
        out.append(t)
    return out


def _pcts(lat: list[float]) -> dict:
    lat = sorted(lat)
    return {"p50_latency_ms": round(1e3 * statistics.median(lat), 1),
            "p90_latency_ms": round(1e3 * lat[int(0.9 * (len(lat) - 1))], 1),
            "p99_latency_ms": round(1e3 * lat[int(0.99 * (len(lat) - 1))], 1)}


def _questions(kind: str, n: int) -> list[str]:
    from docqa_amd.text.synthetic import synthetic_questions, synthetic_unique_questions

    return synthetic_unique_questions(n, seed=77) if kind == "unique" else synthetic_questions(n, seed=77)


def _engine_counters(text: str) -> dict:
    """The continuous scheduler's counters from the llm-qa Prometheus text."""
    out = {}
    for line in text.splitlines():
        if line.startswith("llm_qa_engine_"):
            k, v = line.split()
            out[k[len("llm_qa_engine_"):]] = float(v)
    return out


def _server_split(text: str) -> dict:
    """Server-side latency split (median over the service's recent window): arrival -> prep
    batch start, prep batch duration, engine time, prep batch size."""
    out = {}
    for line in text.splitlines():
        for k in ("ask_queue_s", "ask_prep_batch_s", "ask_engine_s", "ask_latency_s", "ask_batch_size"):
            if line.startswith(f'llm_qa_{k}{{quantile="0.5"}}'):
                out[k + "_p50"] = round(float(line.split()[-1]), 4)
    return out


def run_launch(a, mode: str) -> list[dict]:
    """Start the service launcher, drive it over HTTP at each offered rate, stop it."""
    import asyncio
    import shutil
    import tempfile


    port = 8001 + a.port_offset
    work = tempfile.mkdtemp(prefix="docqa_serving_bench_")   # fresh index / documents DB per run
    env = dict(os.environ, INDEX_DIR=work, DATABASE_URL=f"sqlite:///{work}/documents.db", UPLOAD_DIR=work,
               MAX_NEW_TOKENS=str(a.max_new_tokens), MAX_BATCH=str(a.max_batch), DOCQA_SERVING=mode,
               TEMPERATURE="0", HSA_ENABLE_IPC_MODE_LEGACY="0", STOP_ON_EOS="0" if a.ignore_eos else "1",
               # the server log must survive a crash of the service (no block-buffered stdout)
               PYTHONUNBUFFERED="1", PYTHONFAULTHANDLER="1")
    env.setdefault("PYTHONPATH", str(ROOT))
    cmd = [sys.executable, "-m", "docqa_amd.services.launch", "--services", "indexer,qa",
           "--llm", a.llm, "--device", a.device, "--port-offset", str(a.port_offset),
           "--preload-notes", str(a.notes), "--gpus", str(a.gpus), "--tp", str(a.tp),
           "--kv-mem-fraction", str(a.kv_mem_fraction)]
    if a.tiny:
        cmd.append("--tiny")
    if a.launch_prefix:        # e.g. a rocprofv3 kernel trace of the service process
        import shlex

        cmd = shlex.split(a.launch_prefix) + cmd
    log = open(a.server_log, "w") if a.server_log else subprocess.DEVNULL
    proc = subprocess.Popen(cmd, cwd=str(ROOT), env=env, stdout=log, stderr=subprocess.STDOUT,
                            start_new_session=True)
    qs = _questions(a.questions, a.warmup + a.requests * len(a.rates))
    url = f"http://127.0.0.1:{port}/ask/"
    murl = f"http://127.0.0.1:{port}/metrics"

    async def drive() -> list[dict]:
        # aiohttp, not httpx: at 160+ requests/s an httpx AsyncClient saturates this process's
        # core and sends late, which spread the arrivals the service saw over ~3x the
        # schedule (measured: every request reached the engine alone, 1.8k decode steps for
        # 600 requests vs 750 in-process).  Latency counts from the SCHEDULED arrival (open
        # loop: a late send is charged, not hidden); send lag is reported separately.
        import aiohttp

        conn = aiohttp.TCPConnector(limit=4 * a.max_batch, keepalive_timeout=60)
        async with aiohttp.ClientSession(connector=conn, timeout=aiohttp.ClientTimeout(total=900)) as cl:
            async def post(q: str):
                async with cl.post(url, json={"question": q}) as r:
                    return r.status, (await r.json() if r.status == 200 else None)

            async def metrics_text() -> str:
                async with cl.get(murl) as r:
                    return await r.text()

            t_dead = time.perf_counter() + a.start_timeout
            while True:                       # ready = the index answers a real question
                if proc.poll() is not None:
                    raise RuntimeError(f"launcher exited with {proc.returncode}")
                try:
                    st, _ = await post(qs[0])
                    if st == 200:
                        break
                except aiohttp.ClientError:
                    pass
                if time.perf_counter() > t_dead:
                    raise TimeoutError("service did not become ready")
                waited = a.start_timeout - (t_dead - time.perf_counter())
                if int(waited) % 30 == 0:
                    print(f"[bench_serving] waiting for the service ({waited:.0f} s)", file=sys.stderr, flush=True)
                await asyncio.sleep(1.0)
            # warm-up: prefix cache of the fixed prompt text, connection pool
            rs = await asyncio.gather(*[post(q) for q in qs[1:a.warmup]])
            assert all(st == 200 for st, _ in rs), [st for st, _ in rs if st != 200][:4]
            results = []
            for ri, rate in enumerate(a.rates):
                batch_q = qs[a.warmup + ri * a.requests:a.warmup + (ri + 1) * a.requests]
                lat, lags, dones, errors, empty, retried = [], [], [], 0, 0, 0
                sched = _arrivals(a.requests, rate)
                c0 = _engine_counters(await metrics_text())
                t0 = time.perf_counter()

                async def one(at: float, q: str):
                    nonlocal errors, empty, retried
                    delay = t0 + at - time.perf_counter()
                    if delay > 0:
                        await asyncio.sleep(delay)
                    lags.append(time.perf_counter() - (t0 + at))
                    for attempt in range(2):
                        try:
                            st, body = await post(q)
                            break
                        except (aiohttp.ServerDisconnectedError, aiohttp.ClientOSError):
                            # a pooled keep-alive connection the server closed as it was reused
                            if attempt:
                                raise
                            retried += 1
                    if st != 200:
                        errors += 1
                    elif not body.get("answer"):
                        # no text: EOS first (stop_on_eos), or -- with --ignore-eos, every answer
                        # decoding max_new_tokens (engine counters below) -- a random-init model's
                        # tokens that all detokenise to nothing (ids past the tokenizer's vocab)
                        empty += 1
                    lat.append(time.perf_counter() - (t0 + at))
                    dones.append(time.perf_counter() - t0)

                async def progress():
                    # a line every 15 s: a live run is visibly alive (and a wedged one visibly stuck)
                    while True:
                        await asyncio.sleep(15.0)
                        print(f"[bench_serving] rate {rate}: {len(lat)}/{a.requests} done, errors {errors}, "
                              f"{time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

                pt = asyncio.create_task(progress())
                try:
                    await asyncio.wait_for(
                        asyncio.gather(*[one(at, q) for at, q in zip(sched, batch_q)]),
                        timeout=a.run_timeout)
                finally:
                    pt.cancel()
                wall = time.perf_counter() - t0
                mtext = await metrics_text()
                c1 = _engine_counters(mtext)
                lags.sort()
                # steady state: completions between the first completion and the last
                # scheduled arrival (the ramp before the first answer and the drain after the
                # last arrival excluded), per second of that window
                w0, w1 = min(dones), sched[-1]
                steady = (round(sum(w0 <= d <= w1 for d in dones) / (w1 - w0), 2) if w1 - w0 > 1.0 else None)
                results.append({"rate": rate, "lat": lat, "wall": wall, "errors": errors, "steady": steady,
                                "steady_window_s": round(max(0.0, w1 - w0), 2),
                                "empty_answers": empty, "retried_connections": retried,
                                "send_lag_ms_p50": round(1e3 * lags[len(lags) // 2], 2),
                                "send_lag_ms_max": round(1e3 * lags[-1], 2),
                                "server": _server_split(mtext),
                                "engine": {k: int(c1[k] - c0.get(k, 0)) for k in c1}})
            return results

    try:
        runs = asyncio.run(drive())
    finally:
        try:
            os.killpg(proc.pid, signal.SIGINT)
            proc.wait(timeout=60)
        except (subprocess.TimeoutExpired, ProcessLookupError):
            try:
                os.killpg(proc.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            proc.wait()
        shutil.rmtree(work, ignore_errors=True)
    return [{"metric": "serving_qa_queries_per_sec", "entry": "services.launch (HTTP POST /ask/)",
             "mode": mode, "offered_rate": res["rate"], "value": round(a.requests / res["wall"], 2),
             "unit": "queries/s", "steady_state_qps": res["steady"], "steady_window_s": res["steady_window_s"],
             **_pcts(res["lat"]), "errors": res["errors"],
             "empty_answers": res["empty_answers"], "retried_connections": res["retried_connections"],
             "server_split_p50": res["server"], "send_lag_ms_p50": res["send_lag_ms_p50"],
             "send_lag_ms_max": res["send_lag_ms_max"],
             "requests": a.requests, "max_new_tokens": a.max_new_tokens, "max_batch": a.max_batch,
             "ignore_eos": a.ignore_eos,
             # measured by the engine: tokens emitted, and answers that stopped before
             # max_new_tokens (0 with --ignore-eos: every answer decodes the full length)
             "gen_tokens_per_s": (round(res["engine"].get("generated_tokens", 0) / res["wall"], 1)
                                  if "generated_tokens" in res["engine"] else None),
             "tokens_per_answer": (round(res["engine"]["generated_tokens"] / max(1, res["engine"].get("completed", 0)), 2)
                                   if "generated_tokens" in res["engine"] else None),
             "answers_short_of_max_new_tokens": res["engine"].get("completed_short"),
             "gpus": a.gpus, "tp": a.tp, "llm": "tiny" if a.tiny else a.llm, "notes": a.notes,
             "questions": a.questions, "dtype": "bf16" if a.device != "cpu" else "fp32",
             "data": "synthetic questions and notes, random-init weights", "wall_s": round(res["wall"], 2),
             "scheduler": res["engine"]} for res in runs]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rate", default="80", help="mean arrivals per second (launch entry: a comma list, "
                    "run one after another on the same service)")
    ap.add_argument("--requests", type=int, default=600)
    ap.add_argument("--max-new-tokens", type=int, default=128)
    ap.add_argument("--max-batch", type=int, default=128)
    ap.add_argument("--modes", default="continuous,batch")
    ap.add_argument("--llm", default="llama3-8b")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--entry", choices=("launch", "inproc"), default="launch")
    ap.add_argument("--questions", choices=("unique", "repeat"), default="unique")
    ap.add_argument("--warmup", type=int, default=64)
    ap.add_argument("--gpus", type=int, default=1, help="launch entry: GPUs of the service")
    ap.add_argument("--tp", type=int, default=1, help="launch entry: tensor-parallel size")
    ap.add_argument("--notes", type=int, default=1000, help="launch entry: synthetic notes indexed at start")
    ap.add_argument("--port-offset", type=int, default=20000)
    ap.add_argument("--kv-mem-fraction", type=float, default=0.8)
    ap.add_argument("--start-timeout", type=float, default=900.0)
    ap.add_argument("--run-timeout", type=float, default=600.0, help="launch entry: seconds per offered rate")
    ap.add_argument("--tiny", action="store_true", help="tiny random models (CPU functional run)")
    ap.add_argument("--ignore-eos", action="store_true",
                    help="decode every answer to --max-new-tokens (STOP_ON_EOS=0), as bench.py does: random "
                         "weights otherwise end ~13 %% of answers at the first token")
    ap.add_argument("--server-log", default="", help="file for the launcher's output")
    ap.add_argument("--launch-prefix", default="", help="launch entry: command prepended to the service "
                    "launcher (e.g. 'rocprofv3 --kernel-trace -d DIR -o run --output-format csv --')")
    a = ap.parse_args()
    a.rates = [float(x) for x in a.rate.split(",")]
    a.rate = a.rates[0]
    if a.entry == "launch":
        for mode in a.modes.split(","):
            for out in run_launch(a, mode):
                print(json.dumps(out), flush=True)
        return

    import torch

    from docqa_amd import ops
    from docqa_amd.config import Settings
    from docqa_amd.pipeline.builder import StackConfig, build_stack
    from docqa_amd.services.qa import ContinuousBatcher, DynamicBatcher
    from docqa_amd.utils.metrics import Metrics

    cuda = a.device == "cuda"
    if cuda:
        assert ops.load_native()
    pipe, _ = build_stack(StackConfig(llm=a.llm, max_batch=a.max_batch, max_context=2048,
                                      use_graphs=cuda), device=a.device, log=lambda *x: None)
    qs = _questions(a.questions, a.requests + a.warmup)
    for mode in a.modes.split(","):
        st = Settings()
        st.max_new_tokens = a.max_new_tokens
        st.max_batch = a.max_batch
        st.temperature = 0.0
        st.stop_on_eos = not a.ignore_eos
        cls = ContinuousBatcher if mode == "continuous" else DynamicBatcher
        b = cls(pipe, st, Metrics("bench"))
        # warm-up: capture graphs / tune for the buckets this load will hit
        if mode == "continuous":
            b.engine.warmup()
        for f in [b.submit("ask", q) for q in qs[:a.warmup]]:
            f.result(timeout=600)
        es = pipe.engine.stats
        ce = getattr(b, "engine", None)
        s0 = (es.prefill_s, es.decode_s, es.generated_tokens, getattr(ce, "steps", 0),
              getattr(ce, "preempted", 0), getattr(ce, "kv_blocked", 0))
        arrivals = _arrivals(a.requests, a.rate)
        futs, t0 = [], time.perf_counter()
        for at, q in zip(arrivals, qs[a.warmup:]):
            now = time.perf_counter() - t0
            if at > now:
                time.sleep(at - now)
            futs.append((time.perf_counter(), b.submit("ask", q)))
        lat = []
        for ts, f in futs:
            f.result(timeout=900)
        t_end = time.perf_counter()
        # latency = resolve time - submit time (futures record completion via callbacks)
        lat = sorted(v for v in b.metrics.values("ask_latency_s")[-a.requests:])
        b.stop()
        s1 = (es.prefill_s, es.decode_s, es.generated_tokens, getattr(ce, "steps", 0),
              getattr(ce, "preempted", 0), getattr(ce, "kv_blocked", 0))
        out = {"metric": "serving_qa_queries_per_sec", "entry": "in-process batcher", "mode": mode,
               "offered_rate": a.rate, "value": round(a.requests / (t_end - t0), 2), "unit": "queries/s",
               **_pcts(lat), "questions": a.questions,
               "requests": a.requests, "max_new_tokens": a.max_new_tokens, "max_batch": a.max_batch,
               "ignore_eos": a.ignore_eos,
               "gen_tokens_per_s": (round(a.requests * a.max_new_tokens / (t_end - t0), 1) if a.ignore_eos else None),
               "llm": a.llm, "dtype": "bf16", "data": "synthetic questions, random-init weights",
               "engine_prefill_s": round(s1[0] - s0[0], 2), "engine_decode_s": round(s1[1] - s0[1], 2),
               "decode_steps": s1[3] - s0[3], "wall_s": round(t_end - t0, 2),
               "scheduler": {"preemptions": s1[4] - s0[4], "kv_admission_blocked": s1[5] - s0[5]}}
        print(json.dumps(out), flush=True)
        if cuda:
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
