"""Multi-process spool broker: competing consumers in separate processes each get a
disjoint set of deliveries (atomic-rename claims), acks delete, nack requeues or
dead-letters, and deliveries held by a dead process are redelivered."""
import multiprocessing as mp
import os
import time

from docqa_amd.bus.broker import SpoolBroker


def _consume(root, n_expected, out_q, prefetch):
    b = SpoolBroker(root)
    ch = b.channel()
    ch.queue_declare("work")
    ch.basic_qos(prefetch_count=prefetch)
    got = []

    def cb(c, m, p, body):
        got.append(body.decode())
        c.basic_ack(m.delivery_tag)
        if b.depth("work") == 0:
            c.stop_consuming()

    ch.basic_consume("work", cb)
    deadline = time.time() + 30
    while time.time() < deadline and b.depth("work") > 0:
        ch._dispatch_one(0.05)
    out_q.put(got)


def test_competing_consumers_across_processes(tmp_path):
    root = str(tmp_path / "spool")
    b = SpoolBroker(root)
    for i in range(300):
        b.publish("work", f"m{i}".encode())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_consume, args=(root, 300, q, 4)) for _ in range(3)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    allm = [m for r in res for m in r]
    assert sorted(allm) == sorted(f"m{i}" for i in range(300))   # every message exactly once
    assert len(set(allm)) == 300 and b.depth("work") == 0
    assert not os.listdir(tmp_path / "spool" / "work" / "cur")


def test_nack_requeue_dlq_and_dead_consumer_recovery(tmp_path):
    root = str(tmp_path / "spool")
    b = SpoolBroker(root)
    b.publish("q", b"a")
    b.publish("q", b"b")
    ch = b.channel()
    seen = []

    def cb(c, m, p, body):
        seen.append((body, m.redelivered))
        if body == b"a" and not m.redelivered:
            c.basic_nack(m.delivery_tag, requeue=True)
        elif body == b"b":
            c.basic_nack(m.delivery_tag, requeue=False)
        else:
            c.basic_ack(m.delivery_tag)

    ch.basic_consume("q", cb)
    for _ in range(10):
        ch._dispatch_one(0.05)
    assert (b"a", False) in seen and (b"a", True) in seen and b.get_nowait("q.dlq") == b"b"
    # a delivery claimed by a process that no longer exists goes back to the queue
    b.publish("q", b"c")
    new = tmp_path / "spool" / "q" / "new"
    name = sorted(os.listdir(new))[0]
    os.rename(new / name, tmp_path / "spool" / "q" / "cur" / f"999999999-{name}")
    assert b.depth("q") == 0
    b2 = SpoolBroker(root)
    assert b2.depth("q") == 1 and b2.get_nowait("q") == b"c"


def test_every_broker_exposes_persistent_properties(tmp_path):
    """deid_worker publishes with ``broker.persistent_properties()`` on every backend."""
    from docqa_amd.bus.broker import InProcBroker, SpoolBroker

    for b in (InProcBroker(), SpoolBroker(str(tmp_path / "spool"))):
        assert b.persistent_properties().delivery_mode == 2
