"""Collective health: detect a hung or dead peer in a TP / DP group and fail fast.

SURVEY.md §5.3 asks for "RCCL timeout/abort -> TP-group teardown + re-init".  The
reference has nothing comparable (its only failure handling is the deid reconnect loop,
deid-service/anonymizer.py:89-105).  The MI355X-native shape of it:

  * ``probe(group, timeout_s)`` -- a one-element all-reduce with a bounded wait: True when
    every rank of the group answered, False on timeout / communicator error.  Cheap
    (4 bytes), run between requests, never inside a captured decode graph.
  * ``Watchdog`` -- a heartbeat thread.  The serving loop calls ``beat()`` once per engine
    step; when no beat arrives for ``timeout_s`` while the loop is busy (a collective
    stuck on a dead xGMI peer blocks the host at the next synchronize) the handler runs.
    The default handler exits the process with ``EXIT_COLLECTIVE_HANG``: the group is
    torn down by the process ending and the launcher re-forms it -- ``torchrun
    --max-restarts N`` restarts every rank of the job (fresh rendezvous, fresh RCCL
    communicators), ``services.launch --supervise`` restarts a single-GPU service.
    Re-initialising RCCL inside a process whose communicator hung is not reliable, so the
    process is the unit of recovery.
  * ``reinit(tp_size)`` -- tear down and re-form the groups in-process, for the gloo /
    CPU path and for a planned resize (all ranks alive and agreeing).
"""
from __future__ import annotations

import datetime
import logging
import os
import threading
import time

import torch
import torch.distributed as dist

from . import comm

log = logging.getLogger("docqa.health")

EXIT_COLLECTIVE_HANG = 71


def probe(group=None, timeout_s: float = 10.0) -> bool:
    """True when every rank of ``group`` completes a 1-element all-reduce within
    ``timeout_s``.  Single process: always True."""
    if not dist.is_initialized():
        return True
    s = comm.state()
    cuda = s.backend == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if cuda else torch.device("cpu")
    t = torch.ones(1, dtype=torch.float32, device=dev)
    try:
        work = dist.all_reduce(t, group=group, async_op=True)
        if work.wait(timeout=datetime.timedelta(seconds=timeout_s)) is False:
            return False
        if cuda:
            # the wait orders the stream; bound the host-side completion as well
            ev = torch.cuda.Event()
            ev.record()
            t_end = time.monotonic() + timeout_s
            while not ev.query():
                if time.monotonic() > t_end:
                    return False
                time.sleep(1e-3)
        n = dist.get_world_size(group) if group is not None else dist.get_world_size()
        return int(t.item()) == n
    except Exception as e:  # noqa: BLE001 - timeout, peer gone, aborted communicator
        log.warning("collective probe failed: %s", e)
        return False


def collective_failure(reason: str) -> None:
    """A TP collective failed or a lockstep peer cannot mirror a step: the process's group
    state is undefined, so the process is the unit of recovery -- exit with
    ``EXIT_COLLECTIVE_HANG`` for the launcher (torchrun --max-restarts / launch --supervise)
    to re-form the group.  Tests replace it via ``DOCQA_COLLECTIVE_FAILURE=raise``."""
    log.error("collective failure: %s -- exiting (%d)", reason, EXIT_COLLECTIVE_HANG)
    if os.environ.get("DOCQA_COLLECTIVE_FAILURE", "exit") == "raise":
        raise SystemExit(EXIT_COLLECTIVE_HANG)
    os._exit(EXIT_COLLECTIVE_HANG)


def _exit_handler(stalled_s: float) -> None:
    log.error("no engine step completed for %.1f s: collective presumed hung, exiting (%d)",
              stalled_s, EXIT_COLLECTIVE_HANG)
    os._exit(EXIT_COLLECTIVE_HANG)


class Watchdog:
    """Heartbeat monitor for a serving / benchmark loop.

    ``busy()`` marks the loop as inside a step (only then can a stall be a hang),
    ``beat()`` marks progress, ``idle()`` marks the loop as waiting for work.  The handler
    runs at most once, on the watchdog thread, with the stalled time."""

    def __init__(self, timeout_s: float = 120.0, handler=None, poll_s: float | None = None):
        self.timeout_s = float(timeout_s)
        self.handler = handler or _exit_handler
        self.poll_s = poll_s if poll_s is not None else min(1.0, self.timeout_s / 4)
        self._last = time.monotonic()
        self._busy = False
        self._fired = False
        self._stop = threading.Event()
        self._lock = threading.Lock()
        self._thread = threading.Thread(target=self._run, name="docqa-watchdog", daemon=True)

    @classmethod
    def from_env(cls, var: str = "DOCQA_WATCHDOG_S") -> "Watchdog | None":
        """A started watchdog when ``$var`` is a positive number of seconds, else None."""
        try:
            t = float(os.environ.get(var, "0"))
        except ValueError:
            return None
        return cls(t).start() if t > 0 else None

    def start(self) -> "Watchdog":
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread.is_alive():
            self._thread.join(timeout=5)

    def busy(self) -> None:
        with self._lock:
            if not self._busy:
                self._last = time.monotonic()
            self._busy = True

    def beat(self) -> None:
        with self._lock:
            self._last = time.monotonic()

    def idle(self) -> None:
        with self._lock:
            self._busy = False
            self._last = time.monotonic()

    @property
    def fired(self) -> bool:
        return self._fired

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            with self._lock:
                stalled = time.monotonic() - self._last if self._busy else 0.0
            if stalled > self.timeout_s:
                self._fired = True
                self.handler(stalled)
                return


def reinit(tp_size: int | None = None, backend: str | None = None, timeout_s: int = 600) -> comm.ParallelState:
    """Tear down every process group and re-form them from the same rendezvous env.  All
    ranks must call it (planned TP resize; the gloo path)."""
    global _GEN
    old = comm.state()
    tp = tp_size or old.tp_size
    be = backend or (old.backend if old.backend != "none" else None)
    store = None
    if dist.is_initialized():
        # keep the rendezvous store alive across the teardown and re-form the groups under
        # a fresh key prefix: re-creating the TCP store on MASTER_PORT races with peers
        # still reading the old one
        base = dist.distributed_c10d._get_default_store()
        _GEN += 1
        store = dist.PrefixStore(f"docqa_reinit_{_GEN}", base)
        _STORES.append(base)
    comm.destroy()
    return comm.init_distributed(tp_size=tp, backend=be, timeout_s=timeout_s, store=store)


_GEN = 0
_STORES: list = []       # stores of torn-down groups, kept alive for the re-formed ones
