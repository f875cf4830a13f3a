"""deid-service worker: raw_documents_queue -> de-identify -> clean_documents_queue.

Reference (deid-service/anonymizer.py:50-110):
  * message ``{"doc_id", "text", "metadata"}``; missing doc_id -> "UNKNOWN";
  * output ``{"doc_id", "original_text_masked", "metadata" (passthrough),
    "processed_at": epoch seconds}``, output queue declared durable before publishing,
    then ack;
  * invalid JSON or processing error -> ``nack(requeue=False)`` (here: dead-lettered to
    ``<queue>.dlq`` instead of lost);
  * ``prefetch_count=1``; reconnect every 5 s while the broker is unavailable.
Batching (the MI355X part): the consumer's prefetch window is ``DEID_BATCH_DOCS`` and,
while more raw messages are already queued, the callback only collects them; the batch is
then de-identified by ONE packed NER forward (:meth:`process_messages`: every window of
every document in one varlen encoder pass + the fused token-classification argmax),
published and acked together.  An idle queue flushes at once, so a single document is
not delayed, and a partial batch held while others were queued is flushed by a timer on
the consuming thread after ``DEID_FLUSH_MS`` (default 50 ms) even if no further delivery
arrives (a competing consumer took the rest).  Held messages belong to one channel: a
reconnect drops them (the broker redelivers the unacked ones) rather than acking or
publishing on a dead channel.  A batch whose forward fails is retried one message at a
time, so only a poison message is dead-lettered.
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time

from ..bus.broker import get_broker
from ..config import Settings
from ..deid.engine import DeidEngine

logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(name)s - %(levelname)s - %(message)s")
logger = logging.getLogger("DeID-Service")


class DeidWorker:
    def __init__(self, engine: DeidEngine | None = None, settings: Settings | None = None, broker=None):
        self.st = settings or Settings()
        self.engine = engine or DeidEngine()
        self.broker = broker or get_broker(self.st)
        self.in_q = self.st.raw_queue
        self.out_q = self.st.clean_queue
        self._thread: threading.Thread | None = None
        self._ch = None
        self.processed = 0
        self.batches = 0
        self.batch_docs = max(1, int(getattr(self.st, "deid_batch_docs", 1)))
        self._pending: list = []
        self._pending_t0 = 0.0
        self._timer_armed = False
        self.flush_s = float(os.environ.get("DEID_FLUSH_MS", "50")) / 1e3
        self._depth = getattr(self.broker, "depth", None)

    def clean_message(self, message: dict, masked: str) -> dict:
        return {"doc_id": message.get("doc_id", "UNKNOWN"), "original_text_masked": masked,
                "metadata": message.get("metadata", {}), "processed_at": time.time()}

    def process_messages(self, messages: list[dict]) -> list[dict]:
        masked = self.engine.process_batch([m.get("text", "") or "" for m in messages])
        return [self.clean_message(m, t) for m, t in zip(messages, masked)]

    def callback(self, ch, method, properties, body):
        """Queue consumer: collect while more raw messages are waiting (up to
        ``batch_docs``), then de-identify the batch in one packed forward."""
        if self._pending and self._pending[0][0] is not ch:
            self._pending = []          # held on a channel that is gone: redelivered by the broker
        if not self._pending:
            self._pending_t0 = time.monotonic()
        self._pending.append((ch, method, body))
        waiting = self._depth(self.in_q) if self._depth is not None else 0
        if waiting > 0 and len(self._pending) < self.batch_docs:
            if not self._timer_armed and hasattr(ch, "call_later"):
                self._timer_armed = True
                ch.call_later(self.flush_s, self._flush_stale)
            return
        batch, self._pending = self._pending, []
        self._flush(batch)

    def _flush_stale(self) -> None:
        """Timer (consuming thread): flush a partial batch that has waited ``flush_s``;
        re-arm while a younger one is still being collected."""
        self._timer_armed = False
        if not self._pending:
            return
        age = time.monotonic() - self._pending_t0
        ch = self._pending[0][0]
        if age >= self.flush_s * 0.999:
            batch, self._pending = self._pending, []
            self._flush(batch)
        elif hasattr(ch, "call_later"):
            self._timer_armed = True
            ch.call_later(self.flush_s - age, self._flush_stale)

    def _flush(self, batch: list) -> None:
        good = []
        for ch, method, body in batch:
            try:
                message = json.loads(body)
                if not isinstance(message, dict):
                    raise json.JSONDecodeError("not an object", str(body)[:40], 0)
                good.append((ch, method, message, body))
            except json.JSONDecodeError:
                logger.error("invalid message (not JSON)")
                ch.basic_nack(delivery_tag=method.delivery_tag, requeue=False)
        if not good:
            return
        for _, _, m, _ in good:
            logger.info("[->] doc %s (%d chars)", m.get("doc_id", "UNKNOWN"), len(m.get("text", "") or ""))
        try:
            outs = self.process_messages([m for _, _, m, _ in good])
        except Exception as e:  # noqa: BLE001 - isolate the poison message: one at a time
            if len(good) == 1:
                ch, method, _, _ = good[0]
                logger.error("processing error: %s", e)
                ch.basic_nack(delivery_tag=method.delivery_tag, requeue=False)
                return
            for ch, method, _, body in good:
                self._flush([(ch, method, body)])
            return
        self.batches += 1
        for (ch, method, m, _), out in zip(good, outs):
            try:
                ch.queue_declare(queue=self.out_q, durable=True)
                ch.basic_publish(exchange="", routing_key=self.out_q, body=json.dumps(out),
                                 properties=self.broker.persistent_properties())
                ch.basic_ack(delivery_tag=method.delivery_tag)
                self.processed += 1
                logger.info("[<-] doc %s anonymised -> %s", m.get("doc_id", "UNKNOWN"), self.out_q)
            except Exception as e:  # noqa: BLE001
                logger.error("processing error: %s", e)
                ch.basic_nack(delivery_tag=method.delivery_tag, requeue=False)

    def run_forever(self, retry_s: float = 5.0) -> None:
        while True:
            ch = None
            try:
                ch = self.broker.channel()
                self._ch = ch
                # messages held on the previous channel are unacked there: the broker
                # redelivers them, so never ack / publish them through a dead channel
                self._pending, self._timer_armed = [], False
                ch.queue_declare(queue=self.in_q, durable=True)
                # the reference's prefetch 1 unless this broker can report queue depth (then
                # a window of batch_docs lets the callback drain a burst into one forward)
                ch.basic_qos(prefetch_count=self.batch_docs if self._depth is not None else 1)
                ch.basic_consume(queue=self.in_q, on_message_callback=self.callback)
                logger.info("DeID worker consuming %s", self.in_q)
                ch.start_consuming()
                return
            except KeyboardInterrupt:
                return
            except Exception as e:  # noqa: BLE001 - broker unavailable: retry
                logger.warning("broker unavailable (%s); retrying in %.0fs", e, retry_s)
                self._close_channel(ch)
                ch = None
                time.sleep(retry_s)
            finally:
                self._close_channel(ch)

    @staticmethod
    def _close_channel(ch) -> None:
        """Close a consumer channel (and, under AMQP, its connection) before reconnecting."""
        if ch is None:
            return
        try:
            ch.close()
        except Exception:  # noqa: BLE001 - already broken
            pass

    def start(self) -> "DeidWorker":
        self._thread = threading.Thread(target=self.run_forever, name="deid-worker", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        if self._ch is not None:
            self._ch.stop_consuming()
