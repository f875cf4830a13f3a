"""Collective health (parallel/health.py): the heartbeat watchdog, the bounded-wait
collective probe against a live and a stalled peer (gloo, 2 ranks), and in-process group
re-initialisation.  SURVEY.md §5.3: RCCL timeout/abort -> teardown + re-init."""
import json
import os
import socket
import time

import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_watchdog_fires_only_when_busy_and_stalled():
    from docqa_amd.parallel.health import Watchdog

    fired = []
    wd = Watchdog(0.2, handler=fired.append, poll_s=0.02).start()
    try:
        wd.idle()
        time.sleep(0.4)
        assert not fired, "an idle loop is not a hang"
        wd.busy()
        for _ in range(8):          # beating steps keep it quiet
            time.sleep(0.05)
            wd.beat()
        assert not fired
        time.sleep(0.5)             # a step that never returns
        assert len(fired) == 1 and fired[0] > 0.2 and wd.fired
    finally:
        wd.stop()


def test_watchdog_from_env(monkeypatch):
    from docqa_amd.parallel.health import Watchdog

    monkeypatch.setenv("DOCQA_WATCHDOG_S", "0")
    assert Watchdog.from_env() is None
    monkeypatch.setenv("DOCQA_WATCHDOG_S", "30")
    wd = Watchdog.from_env()
    assert wd is not None and wd.timeout_s == 30
    wd.stop()


def _worker(rank, world, port, out_dir):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import torch.distributed as dist

    from docqa_amd.parallel import comm, health

    comm.init_distributed(tp_size=2, backend="gloo", timeout_s=60)
    res = {"live": health.probe(timeout_s=20)}
    dist.barrier()
    if rank == 0:
        t = time.monotonic()
        res["stalled"] = health.probe(timeout_s=1.0)    # rank 1 is not participating
        res["stalled_s"] = time.monotonic() - t
    else:
        time.sleep(6.0)   # longer than the bounded probe may take on a loaded CI host
    if rank == 1:
        health.probe(timeout_s=20)                      # drain rank 0's pending all-reduce
    st = health.reinit(tp_size=1)
    res["reinit_tp"] = st.tp_size
    res["after_reinit"] = health.probe(timeout_s=20)
    with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
        json.dump(res, f)
    comm.destroy()


def test_probe_detects_stalled_peer_and_reinit(tmp_path):
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    r0 = json.loads((tmp_path / "r0.json").read_text())
    r1 = json.loads((tmp_path / "r1.json").read_text())
    assert r0["live"] and r1["live"]
    # the 1 s probe gave up before the peer (asleep 6 s) could have answered it
    assert r0["stalled"] is False and r0["stalled_s"] < 5.0
    assert r0["reinit_tp"] == 1 and r0["after_reinit"] and r1["after_reinit"]
