"""Online serving benchmark for llm-qa: open-loop Poisson arrivals of clinical questions
into the service's scheduler (RAG embed + kNN + prompt + Llama-3-8B generation), the
continuous-batching scheduler (engine/scheduler.py) against the static dynamic batcher.
Reports completed queries/s and per-request latency percentiles (arrival -> answer).
Synthetic questions, random-init weights.  One JSON line per mode."""
from __future__ import annotations

import argparse
import json
import random
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rate", type=float, default=80.0, help="mean arrivals per second")
    ap.add_argument("--requests", type=int, default=600)
    ap.add_argument("--max-new-tokens", type=int, default=128)
    ap.add_argument("--max-batch", type=int, default=128)
    ap.add_argument("--modes", default="continuous,batch")
    ap.add_argument("--llm", default="llama3-8b")
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()

    import torch

    from docqa_amd import ops
    from docqa_amd.config import Settings
    from docqa_amd.pipeline.builder import StackConfig, build_stack
    from docqa_amd.services.qa import ContinuousBatcher, DynamicBatcher
    from docqa_amd.text.synthetic import synthetic_questions
    from docqa_amd.utils.metrics import Metrics

    cuda = a.device == "cuda"
    if cuda:
        assert ops.load_native()
    pipe, _ = build_stack(StackConfig(llm=a.llm, max_batch=a.max_batch, max_context=2048,
                                      use_graphs=cuda), device=a.device, log=lambda *x: None)
    qs = synthetic_questions(a.requests + 64, seed=77)
    for mode in a.modes.split(","):
        st = Settings()
        st.max_new_tokens = a.max_new_tokens
        st.max_batch = a.max_batch
        st.temperature = 0.0
        cls = ContinuousBatcher if mode == "continuous" else DynamicBatcher
        b = cls(pipe, st, Metrics("bench"))
        # warm-up: capture graphs / tune for the buckets this load will hit
        if mode == "continuous":
            b.engine.warmup()
        for f in [b.submit("ask", q) for q in qs[:64]]:
            f.result(timeout=600)
        es = pipe.engine.stats
        s0 = (es.prefill_s, es.decode_s, es.generated_tokens, getattr(getattr(b, "engine", None), "steps", 0))
        rng = random.Random(0)
        t, arrivals = 0.0, []
        for _ in range(a.requests):
            t += rng.expovariate(a.rate)
            arrivals.append(t)
        futs, t0 = [], time.perf_counter()
        for at, q in zip(arrivals, qs[64:]):
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
        s1 = (es.prefill_s, es.decode_s, es.generated_tokens, getattr(getattr(b, "engine", None), "steps", 0))
        out = {"metric": "serving_qa_queries_per_sec", "mode": mode, "offered_rate": a.rate,
               "value": round(a.requests / (t_end - t0), 2), "unit": "queries/s",
               "p50_latency_ms": round(1e3 * statistics.median(lat), 1),
               "p90_latency_ms": round(1e3 * lat[int(0.9 * (len(lat) - 1))], 1),
               "p99_latency_ms": round(1e3 * lat[int(0.99 * (len(lat) - 1))], 1),
               "requests": a.requests, "max_new_tokens": a.max_new_tokens, "max_batch": a.max_batch,
               "llm": a.llm, "dtype": "bf16", "data": "synthetic questions, random-init weights",
               "engine_prefill_s": round(s1[0] - s0[0], 2), "engine_decode_s": round(s1[1] - s0[1], 2),
               "decode_steps": s1[3] - s0[3], "wall_s": round(t_end - t0, 2)}
        print(json.dumps(out), flush=True)
        if cuda:
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
