"""Failure surfacing of the TP collectives: the IPC
all-reduce records WHICH peer was late in a device error word instead of hanging; every
engine step copies that word behind its kernels and raises ``CollectiveError`` after its
own host sync, so a late or dead peer fails the step instead of returning garbage tokens;
the serving loop hands such a failure to parallel/health.py (exit 71 for the launcher);
a lockstep leader whose step fails tells its followers to drop their running set; the
custom all-reduce's setup decision is collective.  All on CPU: the device word is stubbed."""
import concurrent.futures as cf
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
from docqa_amd.engine.scheduler import ContinuousEngine
from docqa_amd.models.llama import LlamaConfig, LlamaModel
from docqa_amd.parallel import comm
from docqa_amd.parallel.custom_ar import CollectiveError, CustomAllReduce


def _model(seed=7):
    cfg = LlamaConfig(name="tiny-gqa4", vocab_size=4096, hidden=256, intermediate=512, layers=2,
                      heads=8, kv_heads=2, head_dim=128, max_position=2048, bos_token_id=1, eos_token_id=2)
    return LlamaModel(cfg, device="cpu", dtype=torch.float32, seed=seed)


class _StubAR:
    """Stands in for CustomAllReduce: the 'device' error word is a CPU tensor."""

    def __init__(self):
        self.err = torch.zeros(1, dtype=torch.int32)

    def snapshot(self):
        return self.err.clone()

    def raise_if(self, snap):
        if snap is not None and int(snap[0]):
            raise CollectiveError(CustomAllReduce.describe(int(snap[0])))


def _word(peer, phase, epoch):
    return 1 | (peer << 1) | (phase << 4) | (epoch << 8)


def test_error_word_names_the_late_peer():
    msg = CustomAllReduce.describe(_word(5, 1, 1234))
    assert "rank 5" in msg and "phase 1" in msg and "epoch 1234" in msg
    ar = _StubAR()
    ar.raise_if(torch.zeros(1, dtype=torch.int32))           # clean word: no raise
    with pytest.raises(CollectiveError, match="rank 3"):
        ar.raise_if(torch.tensor([_word(3, 0, 7)], dtype=torch.int32))


def test_batch_collect_raises_instead_of_returning_tokens(monkeypatch):
    stub = _StubAR()
    monkeypatch.setattr(comm, "_CUSTOM_AR", stub)
    eng = LLMEngine(_model(), max_batch=4, max_context=256, block_size=16, use_graphs=False)
    p = SamplingParams(max_new_tokens=4, stop_on_eos=False)
    ok = eng.generate([[5, 6, 7, 8]], p)                    # clean word: tokens come back
    assert len(ok[0]) == 4
    stub.err[0] = _word(1, 0, 42)                           # a peer misses a call
    with pytest.raises(CollectiveError, match="rank 1"):
        eng.generate([[5, 6, 7, 8]], p)
    if eng.tail is not None:
        eng.tail.clear()                                    # blocks pinned by the token-granular prefix cache
    st = eng.kv.allocator.stats()                           # the batch's blocks were still freed
    assert st["free"] + st["evictable"] == eng.kv.num_blocks


def test_serving_loop_fails_requests_and_takes_the_exit_path(monkeypatch):
    stub = _StubAR()
    monkeypatch.setattr(comm, "_CUSTOM_AR", stub)
    eng = LLMEngine(_model(), max_batch=4, max_context=256, block_size=16, use_graphs=False)
    ce = ContinuousEngine(eng)
    fired = []
    ce.on_collective_error = lambda e: fired.append(e)
    good = ce.submit([3, 4, 5], SamplingParams(max_new_tokens=3, stop_on_eos=False))
    while ce.has_work():
        ce.step()
    assert len(good.result()) == 3
    stub.err[0] = _word(2, 1, 9)
    bad = ce.submit([3, 4, 5, 6], SamplingParams(max_new_tokens=6, stop_on_eos=False))
    ce.start()
    with pytest.raises(Exception):
        bad.result(timeout=60)
    ce._thread.join(timeout=30)                             # the loop stops after the failure
    assert fired and isinstance(fired[0], CollectiveError) and "rank 2" in str(fired[0])
    assert not ce.running


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _agree_worker(rank, port, fail_rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from docqa_amd.parallel.custom_ar import _agree

    q.put((rank, _agree(rank != fail_rank, None, "cpu"), _agree(True, None, "cpu")))
    dist.destroy_process_group()


def test_setup_decision_is_collective():
    """One rank failing its local setup step makes EVERY rank decide 'fall back' (and no
    rank is left waiting in a barrier the failed one skipped)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_agree_worker, args=(r, port, 1, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    got = sorted(q.get(timeout=5) for _ in range(2))
    assert got == [(0, False, True), (1, False, True)]


def _lockstep_worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from docqa_amd.engine.scheduler import Lockstep

    torch.manual_seed(0)
    eng = LLMEngine(_model(), max_batch=4, max_context=256, block_size=16, use_graphs=False)
    ls = Lockstep(None, src=0, leader=rank == 0)
    ce = ContinuousEngine(eng, lockstep=ls)
    p = SamplingParams(max_new_tokens=6, stop_on_eos=False)
    if rank == 1:
        ce.follow()
        q.put((1, len(ce.running), ce.steps))
    else:
        real = ce._decode
        calls = {"n": 0}

        def flaky():
            calls["n"] += 1
            if calls["n"] == 2:                 # the leader's second decode step fails
                raise RuntimeError("injected leader failure")
            real()

        ce._decode = flaky
        ce.start()
        first = ce.submit([5, 6, 7], p)
        with pytest.raises(RuntimeError, match="injected"):
            first.result(timeout=120)
        # after the reset both ranks run the same (empty) set again: a new request succeeds
        second = ce.submit([8, 9, 10, 11], p)
        out = second.result(timeout=120)
        ce.stop()
        ce.stop_followers()
        q.put((0, len(out), ce.steps))
    dist.destroy_process_group()


def test_lockstep_leader_failure_resets_followers():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_lockstep_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=300)
        assert p.exitcode == 0, p.exitcode
    got = dict((r, (a, b)) for r, a, b in (q.get(timeout=5) for _ in range(2)))
    assert got[0][0] == 6                   # the post-reset request finished on the leader
    assert got[1][0] == 0                   # the follower's running set is empty at "stop"
    # the follower mirrored the post-reset request's steps as well (the failed one aside)
    assert got[1][1] >= got[0][1]
