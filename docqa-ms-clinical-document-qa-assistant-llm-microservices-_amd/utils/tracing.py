"""Request / stage tracing (the reference has no timers or spans beyond
``processed_at``).

``span(name, **attrs)`` records wall-clock spans (thread, start, duration, attributes)
into a bounded in-memory ring when tracing is on (``DOCQA_TRACE=1`` or
:func:`enable`), exportable as Chrome/Perfetto trace-event JSON (``/debug/trace`` on the
llm-qa and semantic-indexer services, :func:`dump`).  With ``DOCQA_ROCTX=1`` every span
is also pushed as a ROCTX range (``torch.cuda.nvtx`` is ROCTX on ROCm), so
``rocprofv3 --marker-trace`` lines the service stages up with the HIP kernels they
launched.  Disabled spans cost one attribute check.
"""
from __future__ import annotations

import collections
import contextlib
import json
import os
import threading
import time

_ENABLED = os.environ.get("DOCQA_TRACE", "0") == "1"
_ROCTX = os.environ.get("DOCQA_ROCTX", "0") == "1"
_EVENTS: collections.deque = collections.deque(maxlen=int(os.environ.get("DOCQA_TRACE_EVENTS", "200000")))
_LOCK = threading.Lock()
_T0 = time.perf_counter()


def enable(on: bool = True, roctx: bool | None = None) -> None:
    global _ENABLED, _ROCTX
    _ENABLED = on
    if roctx is not None:
        _ROCTX = roctx


def enabled() -> bool:
    return _ENABLED


def clear() -> None:
    with _LOCK:
        _EVENTS.clear()


def _roctx(push: bool, name: str = "") -> None:
    try:
        import torch

        if push:
            torch.cuda.nvtx.range_push(name)
        else:
            torch.cuda.nvtx.range_pop()
    except Exception:  # noqa: BLE001 - markers are best effort
        pass


@contextlib.contextmanager
def span(name: str, **attrs):
    if not _ENABLED:
        yield
        return
    if _ROCTX:
        _roctx(True, name)
    t = time.perf_counter()
    try:
        yield
    finally:
        d = time.perf_counter() - t
        if _ROCTX:
            _roctx(False)
        with _LOCK:
            _EVENTS.append((name, threading.get_ident(), threading.current_thread().name, t - _T0, d, attrs))


def instant(name: str, **attrs) -> None:
    if _ENABLED:
        with _LOCK:
            _EVENTS.append((name, threading.get_ident(), threading.current_thread().name,
                            time.perf_counter() - _T0, 0.0, attrs))


def events() -> list[dict]:
    with _LOCK:
        evs = list(_EVENTS)
    return [{"name": n, "tid": tid, "thread": tn, "ts_s": ts, "dur_s": d, "args": a}
            for n, tid, tn, ts, d, a in evs]


def chrome_trace() -> dict:
    """Trace-event JSON (chrome://tracing, ui.perfetto.dev)."""
    pid = os.getpid()
    out, names = [], {}
    for e in events():
        names[e["tid"]] = e["thread"]
        ev = {"name": e["name"], "ph": "X" if e["dur_s"] > 0 else "i", "pid": pid, "tid": e["tid"],
              "ts": round(e["ts_s"] * 1e6, 3), "args": {k: _jsonable(v) for k, v in e["args"].items()}}
        if e["dur_s"] > 0:
            ev["dur"] = round(e["dur_s"] * 1e6, 3)
        else:
            ev["s"] = "t"
        out.append(ev)
    for tid, tn in names.items():
        out.append({"name": "thread_name", "ph": "M", "pid": pid, "tid": tid, "args": {"name": tn}})
    return {"traceEvents": out, "displayTimeUnit": "ms"}


def summary() -> dict:
    """Per-span-name count / total / p50 / p99 (seconds)."""
    by: dict[str, list[float]] = collections.defaultdict(list)
    for e in events():
        by[e["name"]].append(e["dur_s"])
    res = {}
    for k, xs in by.items():
        xs.sort()
        res[k] = {"count": len(xs), "total_s": sum(xs), "p50_s": xs[len(xs) // 2],
                  "p99_s": xs[min(len(xs) - 1, int(0.99 * len(xs)))]}
    return res


def dump(path: str) -> str:
    with open(path, "w") as f:
        json.dump(chrome_trace(), f)
    return path


def _jsonable(v):
    if isinstance(v, (int, float, str, bool)) or v is None:
        return v
    return str(v)
