"""Message bus for the asynchronous ingestion pipeline (raw -> deid -> clean -> indexer).

Two interchangeable backends with a pika-shaped channel API (``basic_publish``,
``basic_consume``, ``basic_ack``/``basic_nack``, ``queue_declare``, ``basic_qos``), so
the worker code reads like the reference's (deid-service/anonymizer.py:50-110,
semantic-indexer/indexer.py:112-137):

* :class:`InProcBroker` (default): named durable queues in process, competing
  consumers with ``prefetch_count`` flow control, manual ack, optional append-only
  journal (``journal_dir``) giving at-least-once delivery across restarts (the
  durable-queue + persistent-message semantics of doc-ingestor/processing.py:27,40),
  and a dead-letter queue ``<queue>.dlq`` for ``nack(requeue=False)`` -- the reference
  silently drops poison messages.
* :class:`SpoolBroker` (``DOCQA_BUS=spool``): the same semantics across PROCESSES on
  a shared directory (atomic-rename claims), so each service can run as its own
  process without a broker daemon;
* :class:`AmqpBroker`: RabbitMQ through pika when it is installed (wire-compatible
  JSON bodies, default exchange, ``delivery_mode=2``).
"""
from __future__ import annotations

import base64
import collections
import itertools
import json
import os
import threading
import time
from dataclasses import dataclass
from pathlib import Path
from typing import Callable


@dataclass
class Method:
    delivery_tag: int
    routing_key: str
    redelivered: bool = False


@dataclass
class Properties:
    delivery_mode: int = 2


class _Queue:
    def __init__(self, name: str, durable: bool):
        self.name = name
        self.durable = durable
        self.ready: collections.deque = collections.deque()   # (msg_id, body, redelivered)
        self.cv = threading.Condition()


class InProcChannel:
    """A consumer/publisher handle; ``prefetch_count`` is per channel, like AMQP."""

    def __init__(self, broker: "InProcBroker"):
        self.broker = broker
        self.prefetch = 0
        self._unacked: dict[int, tuple[str, str, bytes]] = {}
        self._consumers: list[tuple[str, Callable]] = []
        self._stop = threading.Event()
        self._lock = threading.Condition()
        self._timers: list[tuple[float, Callable]] = []

    # --- pika-shaped API
    def queue_declare(self, queue: str, durable: bool = True, **_):
        self.broker.declare(queue, durable)
        return queue

    def basic_qos(self, prefetch_count: int = 0, **_):
        self.prefetch = prefetch_count

    def basic_publish(self, exchange: str = "", routing_key: str = "", body=b"", properties=None, **_):
        if isinstance(body, str):
            body = body.encode()
        self.broker.publish(routing_key, body)

    def basic_consume(self, queue: str, on_message_callback: Callable, auto_ack: bool = False, **_):
        self.broker.declare(queue, True)
        self._consumers.append((queue, on_message_callback))

    def basic_ack(self, delivery_tag: int, **_):
        with self._lock:
            q, mid, _ = self._unacked.pop(delivery_tag)
            self._lock.notify_all()
        self.broker._journal_ack(q, mid)

    def basic_nack(self, delivery_tag: int, requeue: bool = True, **_):
        with self._lock:
            q, mid, body = self._unacked.pop(delivery_tag)
            self._lock.notify_all()
        if requeue:
            self.broker._requeue(q, mid, body)
        else:
            self.broker._journal_ack(q, mid)
            self.broker.publish(q + ".dlq", body)

    def call_later(self, delay: float, fn: Callable) -> None:
        """Run ``fn()`` on the consuming thread after ``delay`` seconds (pika's
        ``BlockingConnection.call_later``): consumer-side timers need no locking."""
        self._timers.append((time.monotonic() + delay, fn))

    def _run_timers(self) -> None:
        if not self._timers:
            return
        now = time.monotonic()
        due = [t for t in self._timers if t[0] <= now]
        if due:
            self._timers = [t for t in self._timers if t[0] > now]
            for _, fn in due:
                fn()

    def start_consuming(self):
        """Blocking dispatch loop (one thread per channel, like pika's BlockingChannel)."""
        while not self._stop.is_set():
            self._dispatch_one(timeout=0.02 if self._timers else 0.05)
            self._run_timers()

    def stop_consuming(self):
        self._stop.set()

    def _dispatch_one(self, timeout: float) -> bool:
        with self._lock:
            if self.prefetch and len(self._unacked) >= self.prefetch:
                self._lock.wait(timeout)
                return False
        for queue, cb in self._consumers:
            got = self.broker._get(queue, timeout=timeout / max(1, len(self._consumers)))
            if got is None:
                continue
            mid, body, redelivered = got
            tag = next(self.broker._tags)
            with self._lock:
                self._unacked[tag] = (queue, mid, body)
            cb(self, Method(tag, queue, redelivered), Properties(), body)
            return True
        return False

    def close(self):
        self.stop_consuming()
        with self._lock:
            pending = list(self._unacked.values())
            self._unacked.clear()
        for q, mid, body in pending:  # unacked -> redelivered, as on a dropped AMQP channel
            self.broker._requeue(q, mid, body)


class InProcBroker:
    def __init__(self, journal_dir: str | None = None):
        self._queues: dict[str, _Queue] = {}
        self._lock = threading.Lock()
        self._tags = itertools.count(1)
        self._ids = itertools.count(1)
        self.journal_dir = Path(journal_dir) if journal_dir else None
        self._jlock = threading.Lock()
        if self.journal_dir:
            self.journal_dir.mkdir(parents=True, exist_ok=True)
            self._replay()

    # --- journal: <queue>.log lines {"op": "pub"|"ack", "id": str, "body": b64}
    def _jpath(self, q: str) -> Path:
        return self.journal_dir / f"{q}.log"

    def _journal(self, q: str, rec: dict) -> None:
        if not self.journal_dir:
            return
        with self._jlock, open(self._jpath(q), "a", encoding="utf-8") as f:
            f.write(json.dumps(rec) + "\n")
            f.flush()
            os.fsync(f.fileno())

    def _journal_ack(self, q: str, mid: str) -> None:
        self._journal(q, {"op": "ack", "id": mid})

    def _replay(self) -> None:
        for p in sorted(self.journal_dir.glob("*.log")):
            q = p.stem
            live: dict[str, bytes] = {}
            for line in p.read_text(encoding="utf-8").splitlines():
                try:
                    r = json.loads(line)
                except json.JSONDecodeError:
                    continue  # torn tail write
                if r["op"] == "pub":
                    live[r["id"]] = base64.b64decode(r["body"])
                else:
                    live.pop(r["id"], None)
            qq = self.declare(q, True)
            for mid, body in live.items():
                qq.ready.append((mid, body, True))
            # compact the journal to the live set
            with open(p, "w", encoding="utf-8") as f:
                for mid, body in live.items():
                    f.write(json.dumps({"op": "pub", "id": mid, "body": base64.b64encode(body).decode()}) + "\n")

    # --- queue ops
    def declare(self, name: str, durable: bool = True) -> _Queue:
        with self._lock:
            q = self._queues.get(name)
            if q is None:
                q = self._queues[name] = _Queue(name, durable)
            return q

    def publish(self, queue: str, body: bytes) -> None:
        q = self.declare(queue, True)
        mid = f"{os.getpid()}-{time.time_ns()}-{next(self._ids)}"
        self._journal(queue, {"op": "pub", "id": mid, "body": base64.b64encode(body).decode()})
        with q.cv:
            q.ready.append((mid, body, False))
            q.cv.notify()

    def _requeue(self, queue: str, mid: str, body: bytes) -> None:
        q = self.declare(queue, True)
        with q.cv:
            q.ready.appendleft((mid, body, True))
            q.cv.notify()

    def _get(self, queue: str, timeout: float):
        q = self.declare(queue, True)
        with q.cv:
            if not q.ready:
                q.cv.wait(timeout)
            if not q.ready:
                return None
            return q.ready.popleft()

    def depth(self, queue: str) -> int:
        q = self.declare(queue, True)
        with q.cv:
            return len(q.ready)

    @staticmethod
    def persistent_properties() -> Properties:
        """Message properties for a persistent publish (every in-proc message is)."""
        return Properties(delivery_mode=2)

    def channel(self) -> InProcChannel:
        return InProcChannel(self)

    def get_nowait(self, queue: str):
        """Test helper: pop one ready message body (auto-acked)."""
        got = self._get(queue, 0.0)
        if got is None:
            return None
        self._journal_ack(queue, got[0])
        return got[1]


class SpoolChannel(InProcChannel):
    """Channel of a :class:`SpoolBroker` (same pika-shaped API and flow control)."""

    def close(self):
        self.stop_consuming()
        with self._lock:
            pending = list(self._unacked.values())
            self._unacked.clear()
        for q, mid, body in pending:
            self.broker._requeue(q, mid, body)


class SpoolBroker:
    """Multi-process durable queues on a shared directory (no daemon): one file per
    message, FIFO by name, claimed by an atomic ``rename`` so competing consumers in
    different processes never receive the same delivery.

        <root>/<queue>/new/<id>           ready
        <root>/<queue>/cur/<pid>-<id>     delivered to a consumer process, unacked
        <root>/<queue>/tmp/<id>           being written (renamed into new/ when complete)

    ack deletes the claimed file, ``nack(requeue=True)`` renames it back (marked
    redelivered), ``nack(requeue=False)`` moves it to ``<queue>.dlq``; deliveries held by
    a process that died are re-queued when any process opens the queue.  This is the
    single-node stand-in for RabbitMQ's durable queues + persistent messages + manual ack
    (doc-ingestor/processing.py:27,40; deid-service/anonymizer.py:79-87) that lets every
    service run in its own process, like the reference's start_all.bat, with no broker
    to install."""

    POLL_S = 0.01

    def __init__(self, root: str, fsync: bool = False):
        self.root = Path(root)
        self.root.mkdir(parents=True, exist_ok=True)
        self.fsync = fsync
        self._tags = itertools.count(1)
        self._ids = itertools.count(1)
        self._declared: set[str] = set()
        self._lock = threading.Lock()

    def _dirs(self, q: str):
        base = self.root / q
        return base / "new", base / "cur", base / "tmp"

    def declare(self, name: str, durable: bool = True):
        with self._lock:
            if name in self._declared:
                return name
            self._declared.add(name)
        new, cur, tmp = self._dirs(name)
        for d in (new, cur, tmp):
            d.mkdir(parents=True, exist_ok=True)
        self._recover(name)
        return name

    def _recover(self, q: str) -> None:
        """Re-queue deliveries whose consumer process is gone."""
        new, cur, _ = self._dirs(q)
        for f in cur.iterdir():
            pid_s, _, mid = f.name.partition("-")
            try:
                os.kill(int(pid_s), 0)
                alive = True
            except (ValueError, ProcessLookupError):
                alive = False
            except PermissionError:
                alive = True
            if not alive:
                try:
                    os.rename(f, new / (mid if mid.endswith(".r") else mid + ".r"))
                except FileNotFoundError:
                    pass

    def publish(self, queue: str, body: bytes) -> None:
        self.declare(queue)
        new, _, tmp = self._dirs(queue)
        mid = f"{time.time_ns():020d}-{os.getpid()}-{next(self._ids)}"
        t = tmp / mid
        with open(t, "wb") as f:
            f.write(body)
            if self.fsync:
                f.flush()
                os.fsync(f.fileno())
        os.rename(t, new / mid)

    def _get(self, queue: str, timeout: float):
        self.declare(queue)
        new, cur, _ = self._dirs(queue)
        deadline = time.monotonic() + timeout
        while True:
            for name in sorted(os.listdir(new)):
                claimed = cur / f"{os.getpid()}-{name}"
                try:
                    os.rename(new / name, claimed)
                except FileNotFoundError:
                    continue                      # another consumer won this one
                body = claimed.read_bytes()
                return claimed.name, body, name.endswith(".r")
            if time.monotonic() >= deadline:
                return None
            time.sleep(min(self.POLL_S, max(0.0, deadline - time.monotonic())))

    def _journal_ack(self, queue: str, mid: str) -> None:
        _, cur, _ = self._dirs(queue)
        try:
            os.unlink(cur / mid)
        except FileNotFoundError:
            pass

    def _requeue(self, queue: str, mid: str, body: bytes) -> None:
        new, cur, _ = self._dirs(queue)
        name = mid.partition("-")[2]
        try:
            os.rename(cur / mid, new / (name if name.endswith(".r") else name + ".r"))
        except FileNotFoundError:
            pass

    def depth(self, queue: str) -> int:
        self.declare(queue)
        return len(os.listdir(self._dirs(queue)[0]))

    persistent_properties = staticmethod(InProcBroker.persistent_properties)

    def channel(self) -> SpoolChannel:
        return SpoolChannel(self)

    def get_nowait(self, queue: str):
        got = self._get(queue, 0.0)
        if got is None:
            return None
        self._journal_ack(queue, got[0])
        return got[1]


class _AmqpChannel:
    """A pika channel that owns its BlockingConnection: ``close()`` closes both, so a
    consumer loop (or a failed one, before the reconnect) never leaks a connection."""

    def __init__(self, conn):
        self._conn = conn
        self._ch = conn.channel()

    def __getattr__(self, name):
        return getattr(self._ch, name)

    def call_later(self, delay: float, fn):  # pragma: no cover - needs a broker
        """Timer on the connection's own thread (runs inside ``start_consuming``)."""
        self._conn.call_later(delay, fn)

    def close(self):  # pragma: no cover - needs a broker
        try:
            if self._ch.is_open:
                self._ch.close()
        finally:
            if self._conn.is_open:
                self._conn.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class AmqpBroker:
    """RabbitMQ via pika (only when pika is importable).  ``publish`` opens one connection
    per message, publishes persistently and closes it, like the reference
    (doc-ingestor/processing.py:21-44); ``channel()`` is for long-lived consumers."""

    def __init__(self, host: str = "localhost"):
        try:
            import pika  # noqa: F401
        except ImportError as e:  # pragma: no cover - pika is absent in CI
            raise RuntimeError("AMQP backend requested but pika is not installed") from e
        self.host = host

    @staticmethod
    def persistent_properties():  # pragma: no cover
        import pika

        return pika.BasicProperties(delivery_mode=2)

    def publish(self, queue: str, body: bytes) -> None:  # pragma: no cover
        import pika

        conn = pika.BlockingConnection(pika.ConnectionParameters(host=self.host))
        try:
            ch = conn.channel()
            ch.queue_declare(queue=queue, durable=True)
            ch.basic_publish(exchange="", routing_key=queue, body=body,
                             properties=pika.BasicProperties(delivery_mode=2))
        finally:
            conn.close()

    def channel(self):  # pragma: no cover
        import pika

        return _AmqpChannel(pika.BlockingConnection(pika.ConnectionParameters(host=self.host)))


_default: InProcBroker | None = None
_dlock = threading.Lock()


def get_broker(settings=None):
    """Process-wide broker selected by ``DOCQA_BUS`` (inproc | amqp)."""
    global _default
    from ..config import settings as _s

    st = settings or _s()
    if st.bus_backend == "amqp":
        return AmqpBroker(st.rabbitmq_host)
    if st.bus_backend == "spool":
        return SpoolBroker(st.spool_dir)
    with _dlock:
        if _default is None:
            _default = InProcBroker(st.bus_journal_dir or None)
        return _default


def reset_default_broker() -> None:
    global _default
    with _dlock:
        _default = None
