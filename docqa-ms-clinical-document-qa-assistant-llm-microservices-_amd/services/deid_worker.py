"""deid-service worker: raw_documents_queue -> de-identify -> clean_documents_queue.

Reference (deid-service/anonymizer.py:50-110):
  * message ``{"doc_id", "text", "metadata"}``; missing doc_id -> "UNKNOWN";
  * output ``{"doc_id", "original_text_masked", "metadata" (passthrough),
    "processed_at": epoch seconds}``, output queue declared durable before publishing,
    then ack;
  * invalid JSON or processing error -> ``nack(requeue=False)`` (here: dead-lettered to
    ``<queue>.dlq`` instead of lost);
  * ``prefetch_count=1``; reconnect every 5 s while the broker is unavailable.
Batching: :meth:`DeidWorker.process_messages` de-identifies a list of raw messages with
one packed NER forward on the GPU (used by the batched path and the config-3 bench).
"""
from __future__ import annotations

import json
import logging
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

    def clean_message(self, message: dict, masked: str) -> dict:
        return {"doc_id": message.get("doc_id", "UNKNOWN"), "original_text_masked": masked,
                "metadata": message.get("metadata", {}), "processed_at": time.time()}

    def process_messages(self, messages: list[dict]) -> list[dict]:
        masked = self.engine.process_batch([m.get("text", "") or "" for m in messages])
        return [self.clean_message(m, t) for m, t in zip(messages, masked)]

    def callback(self, ch, method, properties, body):
        try:
            message = json.loads(body)
            doc_id = message.get("doc_id", "UNKNOWN")
            raw = message.get("text", "") or ""
            logger.info("[->] doc %s (%d chars)", doc_id, len(raw))
            out = self.clean_message(message, self.engine.process_text_anonymization(raw))
            ch.queue_declare(queue=self.out_q, durable=True)
            ch.basic_publish(exchange="", routing_key=self.out_q, body=json.dumps(out),
                             properties=self.broker.persistent_properties())
            ch.basic_ack(delivery_tag=method.delivery_tag)
            self.processed += 1
            logger.info("[<-] doc %s anonymised -> %s", doc_id, self.out_q)
        except json.JSONDecodeError:
            logger.error("invalid message (not JSON)")
            ch.basic_nack(delivery_tag=method.delivery_tag, requeue=False)
        except Exception as e:  # noqa: BLE001
            logger.error("processing error: %s", e)
            ch.basic_nack(delivery_tag=method.delivery_tag, requeue=False)

    def run_forever(self, retry_s: float = 5.0) -> None:
        while True:
            ch = None
            try:
                ch = self.broker.channel()
                self._ch = ch
                ch.queue_declare(queue=self.in_q, durable=True)
                ch.basic_qos(prefetch_count=1)
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
