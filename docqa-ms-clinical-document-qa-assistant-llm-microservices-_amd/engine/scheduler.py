"""Continuous (iteration-level) batching on top of :class:`LLMEngine`.

The static path (:meth:`LLMEngine.generate`) runs one batch from prefill to its last
token; a request that arrives meanwhile waits for the whole batch, and a sequence that
stops early (EOS) leaves its slot idle.  Here the decode batch is a set of SLOTS that
requests join and leave between steps:

  * admission: waiting requests are admitted while slots and KV blocks are free (prompt
    + max_new_tokens blocks reserved up front, prompt-prefix cache hits reused), their
    prompts prefilled together (one packed varlen forward, chunked past the token
    budget) and their first tokens sampled;
  * decode: one step for every running slot -- a HIP graph captured per (batch bucket,
    greedy/sampled, cascade) whose buffers are VIEWS of one slot-state tensor set, so
    moving between buckets as the batch grows and shrinks copies nothing;
  * retirement: a slot whose request hit EOS / its token limit frees its blocks, resolves
    its future, and the last slot moves into the hole (device-side row gather) so slots
    stay dense and the smallest bucket covers them;
  * cascade: when every running slot starts with the same cached prompt-prefix blocks
    (the RAG template), the step attends that prefix once for the whole batch
    (csrc/include/docqa_cascade.h);
  * lagged readback: step t's tokens are copied to pinned host memory and read while
    step t+1 already runs, so the GPU never idles on the host's bookkeeping (a finished
    request rides one extra step inside its reserved blocks and that token is dropped);
  * stall-free admission (mixed steps, DOCQA_MIXED_PREFILL=1; off by default): while
    requests decode, new prompts are prefilled in token-budgeted chunks
    (DOCQA_CHUNK_TOKENS) that ride INSIDE the decode step's forward
    (LlamaModel.forward_mixed): every projection makes one weight pass over the decode
    rows and the chunk's tokens together, only attention is split by row kind.  A
    running request never waits for a separate prefill pass and arrivals are admitted the
    step they come (no hold to batch prefills); a prompt longer than the budget is spread
    over several steps, its first token sampled when its last chunk has run.  Mixed steps
    read their tokens one step late like plain steps, so the eager forward's launch work
    overlaps the GPU.  Still measured SLOWER than admission batching over HTTP
    (profiles/r5_serving_async_mixed_ab.log: offered 60 q/s p50 2.05 s vs 1.38 s, offered
    100 79 vs 92 q/s; the synchronous first version: 2.39 s / 78 q/s,
    profiles/r5_serving_mixed_ab.log): every step that carries a chunk is an eager
    ~500-launch forward instead of a graph replay, and a chunk of 2048 tokens holds every
    decode row for its whole prefill, which admission batching amortises over fewer,
    larger passes;
  * admission batching (mixed steps off, the default): under load, requests are admitted in groups
    (>= ``admit_min`` that can join -- waiting AND free slots -- or ``admit_wait_s``
    after the first could), so one prefill pass over the weights serves several new
    requests instead of stalling every decode step.

Reference parity: the reference serves one blocking request at a time
(llm-qa/main.py:111-117); its generator (Ollama) schedules requests internally.
"""
from __future__ import annotations

import collections
import concurrent.futures as cf
import itertools
import os
import threading
import time
from dataclasses import dataclass, field

import torch

from .. import ops
from ..parallel import comm
from ..parallel.custom_ar import CollectiveError
from ..utils import tracing
from .llm_engine import LLMEngine, SamplingParams, _bucket, _DecodeGraph, _prefill_inputs


@dataclass
class Request:
    rid: int
    prompt: list[int]
    params: SamplingParams
    future: cf.Future
    on_token: object = None          # callable(rid, token) for streaming
    out: list[int] = field(default_factory=list)
    blocks: list[int] = field(default_factory=list)
    cached: int = 0
    res: object = None   # the engine Reservation (prefix-copy pins, block keys)
    t_arrival: float = 0.0
    t_first: float = 0.0
    done: bool = False
    # preemption (recompute): generated tokens already folded into ``prompt`` when the
    # request was re-queued, the original prompt length, and the next decode write position
    gen_base: int = 0
    orig_len: int = -1
    pos: int = 0
    preemptions: int = 0
    filled: int = 0      # mixed steps: prompt tokens already in the KV cache


class Lockstep:
    """Keeps the continuous-batching engines of every rank of a tensor-parallel group in
    step: the group leader (TP rank 0, which serves HTTP) owns the request queue and the
    timing-dependent admission decision; before every engine step it broadcasts the
    requests that arrived since the last step and that decision over a CPU (gloo) group.
    Everything else a step does -- KV reservation, prefix-cache hits, prefill, decode,
    retirement on EOS -- is a deterministic function of that input and of the greedy ids,
    which the vocab-parallel argmax makes identical on every rank, so the followers' TP
    forwards always match the leader's.  While idle the leader sends a heartbeat every
    ``heartbeat_s`` so the followers' receive never times out."""

    def __init__(self, group, src: int, leader: bool, heartbeat_s: float = 1.0):
        self.group, self.src, self.leader, self.heartbeat_s = group, src, leader, heartbeat_s
        self.last = time.monotonic()

    def exchange(self, msg=None):
        import torch.distributed as dist

        box = [msg]
        dist.broadcast_object_list(box, src=self.src, group=self.group)
        self.last = time.monotonic()
        return box[0]


class ContinuousEngine:
    def __init__(self, engine: LLMEngine, max_running: int | None = None, lockstep: Lockstep | None = None):
        self.eng = engine
        self.lockstep = lockstep
        self._unsynced: list = []           # lockstep leader: arrivals not yet broadcast
        self.max_running = min(max_running or engine.max_batch, engine.max_batch)
        self.waiting: collections.deque[Request] = collections.deque()
        self.running: list[Request] = []
        self._cv = threading.Condition()
        self._ids = itertools.count()
        self._master = _DecodeGraph(engine, engine.max_batch)
        self._graphs: dict[tuple, _DecodeGraph] = {}
        self._nshared = 0
        self._shared_head: list[int] = []
        self._thread: threading.Thread | None = None
        self._stop = threading.Event()
        self.steps = 0
        # decode over power-of-two slot buckets (padded slots: valid 0); on by default with
        # graphs, settable on CPU to exercise the padded-slot paths of the reference ops
        self.pad_buckets = engine.use_graphs
        self.admit_min = max(1, self.max_running // int(os.environ.get("DOCQA_ADMIT_DIV", "4")))
        self.admit_wait_s = float(os.environ.get("DOCQA_ADMIT_WAIT_MS", "160")) / 1e3
        self._free_t = None                # when a slot last became free with the batch full before
        self._pool = None
        self._pending = None               # (event, pinned host tokens, slot -> request) of the last step
        self._processing = None            # the readback being processed (see _process)
        self._host = None
        self._flip = 0
        self._mhost = None   # mixed steps' pinned token buffers (decode rows + first tokens)
        self._mflip = 0
        # CPU runs read each step's tokens at once; True: lag them by one step as on a GPU
        # (the tests exercise the GPU's readback order on the CPU this way)
        self.lag_cpu = False
        self._version = 0                  # bumped whenever the running set changes
        # KV blocks on demand: admission reserves the prompt + ``reserve_ahead`` generated
        # tokens (not all max_new_tokens), tables grow a block at a time as decode reaches
        # them, and when the pool runs out the youngest running request is preempted and
        # re-queued with its tokens so far appended to its prompt (recompute: its prompt
        # blocks are still in the prefix cache).  DOCQA_PREEMPT=0: reserve everything up
        # front, as before (no preemption ever needed).
        self.preempt = os.environ.get("DOCQA_PREEMPT", "1") == "1"
        self.reserve_ahead = int(os.environ.get("DOCQA_RESERVE_AHEAD", str(engine.block_size)))
        self.preempted = 0
        self.kv_blocked = 0       # admissions deferred because the KV pool was out of blocks
        self.generated = 0        # tokens emitted to requests
        self.completed = 0        # requests finished
        self.completed_short = 0  # ... of them before max_new_tokens (EOS)
        # stall-free admission: prompt chunks ride in the decode step (module docstring)
        self.mixed = os.environ.get("DOCQA_MIXED_PREFILL", "0") == "1"
        self.mixed_hold = os.environ.get("DOCQA_MIXED_HOLD", "0") == "1"
        self.chunk_tokens = max(engine.block_size, int(os.environ.get("DOCQA_CHUNK_TOKENS", "2048")))
        self.prefilling: list[Request] = []   # admitted, prompt partly in the KV cache
        self.mixed_steps = 0

    # ------------------------------------------------------------------ client side
    def submit(self, prompt: list[int], params: SamplingParams | None = None, on_token=None) -> cf.Future:
        params = params or SamplingParams()
        fut: cf.Future = cf.Future()
        if len(prompt) + params.max_new_tokens > self.eng.max_context or not prompt:
            fut.set_exception(ValueError(
                f"prompt+generation {len(prompt) + params.max_new_tokens} exceeds max_context {self.eng.max_context}"))
            return fut
        r = Request(next(self._ids), list(prompt), params, fut, on_token, t_arrival=time.perf_counter())
        with self._cv:
            # a lockstep leader queues arrivals for the next step's broadcast, so the
            # followers see exactly the waiting queue its admission sees
            (self._unsynced if self.lockstep is not None else self.waiting).append(r)
            self._cv.notify()
        return fut

    def has_work(self) -> bool:
        return bool(self.waiting or self.running or self.prefilling or self._pending or self._unsynced)

    def generate(self, prompts: list[list[int]], params: SamplingParams | None = None) -> list[list[int]]:
        """Submit all prompts and drive the scheduler in this thread until they finish."""
        futs = [self.submit(p, params) for p in prompts]
        while not all(f.done() for f in futs):
            self.step()
        return [f.result() for f in futs]

    @torch.inference_mode()
    def warmup(self, buckets: list[int] | None = None, sampled: bool = False) -> None:
        """Capture the decode graphs of every bucket (plain and cascade; greedy, and
        sampled if asked) before serving, so no request pays a capture / GEMM-tuning
        stall mid-stream.  Slots are empty (valid 0): the captured warm-up steps write
        nothing to the KV cache."""
        if not self.eng.use_graphs or self.running:
            return
        bs, b = [], 1
        while b < self.eng.max_batch:
            bs.append(b)
            b *= 2
        bs.append(self.eng.max_batch)
        casc = [False, True] if self.eng.cascade else [False]
        for bp in buckets or bs:
            for greedy in ([True, False] if sampled else [True]):
                for c in casc:
                    g = self._graph(bp, greedy, c)
                    if g.graph is None:
                        if self._pool is None:
                            self._pool = torch.cuda.graph_pool_handle()
                        self.eng._capture(g, self._pool)

    # ------------------------------------------------------------------ serving thread
    def start(self) -> "ContinuousEngine":
        if self._thread is None:
            self._thread = threading.Thread(target=self._serve, name="llm-scheduler", daemon=True)
            self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        with self._cv:
            self._cv.notify()
        if self._thread is not None:
            self._thread.join(timeout=30)
            self._thread = None

    def _serve(self) -> None:
        while not self._stop.is_set():
            with self._cv:
                if not self.has_work():
                    self._cv.wait(timeout=0.1)
                    continue
            try:
                self.step()
            except CollectiveError as e:
                # the TP group's state is undefined: fail the requests, then hand the process
                # to the collective-failure path (parallel/health.py: exit 71, relaunch)
                self._fail_all(e)
                self._reset_followers()
                self.on_collective_error(e)
                return
            except Exception as e:  # noqa: BLE001 - fail the affected requests, keep serving
                self._fail_all(e)
                self._reset_followers()

    def on_collective_error(self, e: Exception) -> None:
        from ..parallel import health

        health.collective_failure(str(e))

    def _reset_followers(self) -> None:
        """Lockstep leader after a failed step: tell the followers to drop their running set
        too, so every rank's next step has the same batch composition (the mirror invariant
        the TP collectives rely on)."""
        ls = self.lockstep
        if ls is not None and ls.leader:
            try:
                ls.exchange(("reset",))
            except Exception:  # noqa: BLE001 - a dead follower: its own exit path handles it
                pass

    def _fail_all(self, e: Exception) -> None:
        lagged = []
        for p in (self._pending, self._processing):
            if p is not None and isinstance(p[0], str):
                lagged += list(p[4])         # a mixed step's completing prompts
        self._pending = self._processing = None
        seen = set()
        for r in self.running + self.prefilling + lagged:
            if id(r) in seen:                # a completing prompt already placed in a slot
                continue
            seen.add(id(r))
            self.eng.kv.allocator.free(r.blocks)
            r.blocks = []
            if not r.future.done():
                r.future.set_exception(e)
        self.running = []
        self.prefilling = []
        self._version += 1
        self._master.valid.zero_()
        self._master.context_lens.zero_()

    # ------------------------------------------------------------------ one iteration
    @torch.inference_mode()
    def step(self) -> None:
        decision = None
        if self.lockstep is not None:
            if not self.lockstep.leader:
                raise RuntimeError("a lockstep follower runs follow(), not step()")
            with self._cv:
                new, self._unsynced = self._unsynced, []
                self.waiting.extend(new)
            decision = self._admission_due()
            try:
                self.lockstep.exchange(("step", [(r.prompt, r.params) for r in new], decision))
            except Exception as e:  # noqa: BLE001 - a follower is gone: the TP group is broken
                raise CollectiveError(f"lockstep broadcast failed: {e!r}") from e
        self._step(decision)

    def _step(self, decision) -> None:
        if self._mixed_due(decision):
            self._mixed_step(decision)
            return
        self._admit(decision)
        if self.running:
            self._decode()
        elif self._pending is not None:
            p, self._pending = self._pending, None
            self._process(p)

    # ------------------------------------------------------------------ lockstep (TP)
    def heartbeat(self) -> None:
        """Lockstep leader, idle: keep the followers' receive alive."""
        ls = self.lockstep
        if ls is not None and ls.leader and time.monotonic() - ls.last >= ls.heartbeat_s:
            ls.exchange(("noop",))

    def stop_followers(self) -> None:
        if self.lockstep is not None and self.lockstep.leader:
            self.lockstep.exchange(("stop",))

    @torch.inference_mode()
    def follow(self) -> None:
        """Lockstep follower loop: mirror every step the leader broadcasts until "stop";
        "reset" (the leader's step failed) drops the running set as the leader did.  A step
        that fails HERE cannot be mirrored back, so the follower exits non-zero: the
        leader's next broadcast then errors instead of its TP collectives hanging."""
        ls = self.lockstep
        while True:
            msg = ls.exchange()
            if msg[0] == "stop":
                return
            if msg[0] == "reset":
                self._fail_all(RuntimeError("leader step failed"))
                continue
            if msg[0] != "step":
                continue
            _, specs, decision = msg
            for prompt, params in specs:
                self.waiting.append(Request(next(self._ids), list(prompt), params, cf.Future(),
                                            t_arrival=time.perf_counter()))
            try:
                self._step(decision)
            except Exception as e:  # noqa: BLE001
                self.on_follower_failure(e)
                return

    def on_follower_failure(self, e: Exception) -> None:
        from ..parallel import health

        health.collective_failure(f"lockstep follower step failed: {e!r}")

    def _take_waiting(self, mixed: bool = False, token_cap: int | None = None) -> list[Request]:
        """Reserve KV blocks for waiting requests while slots are free.  ``mixed``: for the
        chunked-prefill queue -- greedy requests only (a sampled one waits for a plain
        admission), and stop once ``token_cap`` prompt tokens are taken."""
        eng, alloc = self.eng, self.eng.kv.allocator
        admitted, budget = [], 0
        with self._cv:
            while self.waiting and self._occupied() + len(admitted) < self.max_running:
                r = self.waiting[0]
                if mixed and (r.params.temperature > 0 or (token_cap is not None and budget >= token_cap)):
                    break
                if r.orig_len < 0:
                    r.orig_len = len(r.prompt)
                remaining = r.params.max_new_tokens - r.gen_base
                gen = min(remaining, self.reserve_ahead) if self.preempt else remaining
                try:
                    # prefix-cache hits (whole blocks + token-granular rows), fresh blocks
                    res = eng.reserve([r.prompt], r.params, gen_tokens=gen)
                except MemoryError:
                    # can never fit: nothing else holds KV (running rows, prompts being
                    # chunk-prefilled, lagged completions) to free -- fail, don't stall
                    if self._occupied() == 0 and not admitted:
                        need = eng.kv.blocks_for(len(r.prompt) + gen)
                        self.waiting.popleft().future.set_exception(MemoryError(
                            f"request needs {need} KV blocks, the cache has {alloc.num_free()} free"))
                        continue
                    self.kv_blocked += 1
                    break                        # retry after running requests retire
                r.blocks, r.cached, r.res = res.tables[0], res.cached[0], res
                res.tables = []                  # owned by the request from here on
                admitted.append(self.waiting.popleft())
                budget += len(r.prompt) - r.cached
                if budget >= eng.max_prefill_tokens:
                    break
        return admitted

    def _occupied(self) -> int:
        """Decode slots taken or promised: running rows, prompts being chunk-prefilled, and
        prompts whose last chunk ran in the step whose tokens are still to be read (they
        join the running rows when that lagged readback is processed)."""
        lag = len(self._pending[4]) if self._pending is not None and isinstance(self._pending[0], str) else 0
        return len(self.running) + len(self.prefilling) + lag

    def _admission_due(self) -> bool:
        """Whether the waiting requests are admitted at this step (the timing-dependent
        half of admission; a lockstep leader broadcasts it)."""
        if self.mixed and not self.mixed_hold and self.running and self.waiting:
            # chunks ride in the decode steps: admit as soon as a slot is free, no hold
            return self._occupied() < self.max_running
        if self.running and self.waiting:
            # gather a group -- one prefill pass over the weights for several requests --
            # until admit_min requests can join or the first of them has waited
            # admit_wait_s.  Both sides count: under overload the queue is long but slots
            # free up one or two per step as requests finish, and admitting them as they
            # appear ran a near-empty prefill pass every step or two (continuous 114.6 vs
            # static 118.9 q/s at Poisson 140, prefill 29 % of the wall time).
            free = self.max_running - self._occupied()
            now = time.perf_counter()
            if free <= 0:
                self._free_t = None
                return False
            if self._free_t is None:
                self._free_t = now             # a slot just became free
            start = max(self.waiting[0].t_arrival, self._free_t)   # first admissible moment
            if min(len(self.waiting), free) < self.admit_min and now - start < self.admit_wait_s:
                return False
        return True

    def _admit(self, decision: bool | None = None) -> None:
        if decision is None:
            decision = self._admission_due()
        if not decision:
            return
        adm = self._take_waiting()
        if not adm:
            return
        eng, alloc = self.eng, self.eng.kv.allocator
        t0 = time.perf_counter()
        try:
            with tracing.span("sched.admit", seqs=len(adm), tokens=sum(len(r.prompt) - r.cached for r in adm)):
                for r in adm:
                    eng.queue_prefix_copies(r.res)
                greedy = all(r.params.temperature <= 0 for r in adm)
                out = eng._prefill([r.prompt for r in adm], [r.blocks for r in adm], [r.cached for r in adm],
                                   greedy=greedy)
                err = comm.collective_error_snapshot()
                first = out.tolist() if greedy else self._sample_rows(out, [r.params for r in adm])
                comm.raise_on_collective_error(err)
        except CollectiveError:
            for r in adm:
                eng.release(r.res)
                alloc.free(r.blocks)
                r.future.set_exception(RuntimeError("TP collective failed during prefill"))
            raise
        except Exception as e:  # noqa: BLE001
            for r in adm:
                eng.release(r.res)
                alloc.free(r.blocks)
                r.future.set_exception(e)
            return
        eng.register_prefixes([r.prompt for r in adm], [r.blocks for r in adm], [r.res.keys[0] if r.res.keys else None
                                                                                  for r in adm])
        now = time.perf_counter()
        eng.stats.prefill_s += now - t0
        eng.stats.prompt_tokens += sum(len(r.prompt) for r in adm)
        eng.stats.cached_tokens += sum(r.cached for r in adm)
        joined = []
        for r, t in zip(adm, first):
            r.t_first = now
            self._emit(r, t)
            if self._finished(r):
                r.done = True
                self._retire(r)
            else:
                joined.append(r)
        if joined:
            self._place(joined)
        self._update_shared()

    # ------------------------------------------------------------------ mixed steps
    def _mixed_due(self, decision=None) -> bool:
        """A mixed step runs while prompt chunks are pending, or when greedy requests wait
        beside a greedy running batch (sampled decode rows keep the separate prefill).
        ``mixed_hold``: new prompts wait for the admission-batching decision (``decision``,
        the leader's in lockstep) as with mixed steps off, so prompts are prefilled in a
        few large chunks that ride in one decode step each, read back one step late."""
        if not self.mixed:
            return False
        if self.prefilling:
            return True
        due = bool(self.running and self.waiting and self.waiting[0].params.temperature <= 0
                   and all(r.params.temperature <= 0 for r in self.running))
        if due and self.mixed_hold:
            due = self._admission_due() if decision is None else bool(decision)
        return due

    def _mixed_step(self, decision) -> None:
        """One forward over every running slot's next token AND up to ``chunk_tokens`` of
        the pending prompts (LlamaModel.forward_mixed).  Asynchronous like a plain decode
        step: this step's tokens (decode rows + the first tokens of the prompts whose last
        chunk ran) are copied to pinned host memory and read while the NEXT step runs, so
        the eager forward's launch work overlaps the GPU instead of serialising with it
        (the synchronous version lost to admission batching, profiles/r5_serving_mixed_ab.log).
        A prompt that completes here joins the decode slots when its tokens are processed,
        one step later."""
        eng, BS = self.eng, self.eng.block_size
        if decision is None:
            decision = self._admission_due()
        if decision and self.waiting:
            pend = sum(len(r.prompt) - r.filled for r in self.prefilling)
            cap = 2 * self.chunk_tokens - pend
            if cap > 0:
                for r in self._take_waiting(mixed=True, token_cap=cap):
                    eng.queue_prefix_copies(r.res)
                    r.filled = r.cached
                    self.prefilling.append(r)
        if not self.prefilling:
            if self.running:
                self._decode()
            elif self._pending is not None:
                p, self._pending = self._pending, None
                self._process(p)
            return
        self._grow_tables()
        if not self.prefilling:
            # KV pressure re-queued every prefilling prompt (_preempt_youngest): a plain step
            if self.running:
                self._decode()
            return
        t0 = time.perf_counter()
        pieces, budget = [], self.chunk_tokens
        for r in self.prefilling:
            if budget <= 0:
                break
            start = min(r.filled, len(r.prompt) - 1)    # >= 1 token: its logits pick the first
            end = min(len(r.prompt), start + budget)
            pieces.append((r, start, end))
            budget -= end - start
        n = len(self.running)
        dev = eng.device
        g, bp, dmeta = None, 0, None
        if n:
            bp = _bucket(n, eng.max_batch) if self.pad_buckets else n
            fit = self._groups_fit()
            grouped = self._nshared > 0 or eng.group_without_prefix(n, fit)
            g = self._graph(bp, True, grouped, fit)
            if eng.lpt:
                eng.set_order(g, [len(r.prompt) + len(r.out) for r in self.running], key=self._version)
            if grouped and g.groups_fit:
                eng.set_groups(g, [r.blocks for r in self.running],
                               [len(r.prompt) + r.params.max_new_tokens for r in self.running], self._nshared,
                               key=(self._version, self._nshared), ids=[r.rid for r in self.running])
            dmeta = eng._decode_meta(g)
        from ..models.llama import AttnMeta

        ids, pos, slots, cu = _prefill_inputs([r.prompt[:e] for r, _, e in pieces], [r.blocks for r, _, _ in pieces],
                                              [s_ for _, s_, _ in pieces], BS)
        maxb = max(len(r.blocks) for r, _, _ in pieces)
        btab = torch.zeros(len(pieces), maxb, dtype=torch.int32)
        for i, (r, _, _) in enumerate(pieces):
            btab[i, :len(r.blocks)] = torch.tensor(r.blocks, dtype=torch.int32)
        pmeta = AttnMeta(prefill=True, positions=torch.from_numpy(pos).to(dev), slot_mapping=torch.from_numpy(slots).to(dev),
                         cu_seqlens=torch.from_numpy(cu).to(dev), max_len=max(e - s_ for _, s_, e in pieces),
                         block_tables=btab.to(dev),
                         prefix_lens=torch.tensor([s_ for _, s_, _ in pieces], dtype=torch.int32).to(dev))
        done = [i for i, (r, _, e) in enumerate(pieces) if e == len(r.prompt)]
        rows = list(range(bp)) + [bp + int(cu[i + 1]) - 1 for i in done]
        chunk_ids = torch.from_numpy(ids).to(dev)
        input_ids = torch.cat([g.tokens, chunk_ids]) if bp else chunk_ids
        with tracing.span("sched.mixed", running=n, bucket=bp, chunk_tokens=int(cu[-1]), completes=len(done)):
            nxt = eng.model.forward_mixed(input_ids, bp, dmeta, pmeta, eng.kv.caches,
                                          torch.tensor(rows, dtype=torch.long).to(dev))
            if bp:
                ops.decode_advance(nxt[:bp].long().contiguous(), g.out, g.tokens, g.positions, g.context_lens,
                                   g.valid)
        # launch-time bookkeeping: everything that does not need the tokens
        self.steps += 1
        self.mixed_steps += 1
        eng.stats.generated_tokens += n
        snap = list(self.running)
        for r in snap:
            r.pos += 1
        for r, _, e in pieces:
            r.filled = e
        completing = [pieces[i][0] for i in done]
        if completing:
            gone = {id(r) for r in completing}
            self.prefilling = [r for r in self.prefilling if id(r) not in gone]
        k = len(rows)
        if nxt.device.type == "cuda":
            if self._mhost is None or self._mhost[0].dtype != nxt.dtype or self._mhost[0].numel() < k:
                size = max(k, eng.max_batch + self.chunk_tokens)
                self._mhost = [torch.empty(size, dtype=nxt.dtype, pin_memory=True) for _ in range(2)]
            host = self._mhost[self._mflip]
            self._mflip ^= 1
            host[:k].copy_(nxt[:k], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            host, ev = nxt[:k].clone(), None
        pend = ("mixed", ev, host, snap, completing, bp, comm.collective_error_snapshot())
        prev, self._pending = self._pending, pend
        if prev is not None:
            self._process(prev)              # step t-1's tokens while step t runs
        if ev is None and not self.lag_cpu:
            p, self._pending = self._pending, None
            self._process(p)
        eng.stats.decode_s += time.perf_counter() - t0

    def _process_mixed(self, pending) -> None:
        """The lagged readback of a mixed step: decode rows as in :meth:`_process`, then
        the prompts whose last chunk ran -- prefix registration, first token, a decode
        slot (or retirement)."""
        _, ev, host, snap, completing, bp, err = pending
        if ev is not None:
            ev.synchronize()
        comm.raise_on_collective_error(err)
        toks = host[:bp + len(completing)].tolist()
        finished = []
        for r, t in zip(snap, toks[:len(snap)]):
            if r.done:
                continue                      # the extra lagged step of a finished request
            self._emit(r, t)
            if self._finished(r):
                r.done = True
                finished.append(r)
        if finished:
            for r in finished:
                self._retire(r)
            self._compact([i for i, r in enumerate(self.running) if not r.done])
        if completing:
            eng = self.eng
            eng.register_prefixes([r.prompt for r in completing], [r.blocks for r in completing],
                                  [r.res.keys[0] if r.res is not None and r.res.keys else None for r in completing])
            eng.stats.prompt_tokens += sum(len(r.prompt) for r in completing)
            eng.stats.cached_tokens += sum(r.cached for r in completing)
            now = time.perf_counter()
            joined = []
            for r, t in zip(completing, toks[bp:]):
                r.t_first = now
                self._emit(r, t)
                if self._finished(r):
                    r.done = True
                    self._retire(r)
                else:
                    joined.append(r)
            if joined:
                self._place(joined)
        self._update_shared()

    def _place(self, reqs: list[Request]) -> None:
        """Write the decode state of newly joined requests into slots [n, n + k)."""
        m, n, k = self._master, len(self.running), len(reqs)
        maxb = self.eng.max_blocks_per_seq
        bt = torch.zeros(k, maxb, dtype=torch.int32)
        tok = torch.empty(k, dtype=torch.int32)
        pos = torch.empty(k, dtype=torch.int32)
        it = torch.ones(k, dtype=torch.float32)
        tk = torch.zeros(k, dtype=torch.int32)
        tp = torch.ones(k, dtype=torch.float32)
        for i, r in enumerate(reqs):
            bt[i, :len(r.blocks)] = torch.tensor(r.blocks, dtype=torch.int32)
            tok[i] = r.out[-1]
            # the input of the next step sits right after the prompt (+ tokens generated since
            # (re-)admission; gen_base of them are already part of a resumed prompt)
            r.pos = len(r.prompt) + len(r.out) - r.gen_base - 1
            pos[i] = r.pos
            if r.params.temperature > 0:
                it[i], tk[i], tp[i] = 1.0 / r.params.temperature, r.params.top_k, r.params.top_p
            else:
                tk[i] = 1                        # greedy row inside a sampled batch: argmax
        dev = m.tokens.device
        sl = slice(n, n + k)
        m.block_tables[sl].copy_(bt.to(dev, non_blocking=True))
        m.tokens[sl].copy_(tok.to(dev, non_blocking=True))
        m.positions[sl].copy_(pos.to(dev, non_blocking=True))
        m.context_lens[sl].copy_((pos + 1).to(dev, non_blocking=True))
        m.valid[sl].fill_(1)
        m.inv_temp[sl].copy_(it.to(dev, non_blocking=True))
        m.top_k[sl].copy_(tk.to(dev, non_blocking=True))
        m.top_p[sl].copy_(tp.to(dev, non_blocking=True))
        self.running.extend(reqs)
        self._version += 1

    def _sample_rows(self, logits: torch.Tensor, params: list[SamplingParams]) -> list[int]:
        model = self.eng.model
        if all(p.temperature <= 0 for p in params):
            return model.greedy(logits).tolist()
        full = model.full_logits(logits).float()
        dev = full.device
        it = torch.tensor([1.0 / p.temperature if p.temperature > 0 else 1.0 for p in params], device=dev)
        tk = torch.tensor([p.top_k if p.temperature > 0 else 1 for p in params], dtype=torch.int32, device=dev)
        tp = torch.tensor([p.top_p if p.temperature > 0 else 1.0 for p in params], device=dev)
        u = torch.rand(full.shape[0], device=dev)
        return ops.sample(full, it, tk, tp, u).tolist()

    def _graph(self, bp: int, greedy: bool, cascade: bool, fit: bool = True) -> _DecodeGraph:
        fit = fit or self._master.groups_fit
        key = (bp, greedy, cascade, fit)
        g = self._graphs.get(key)
        if g is None:
            g = _DecodeGraph.view_of(self._master, bp)
            g.greedy, g.cascade, g.groups_fit = greedy, cascade, fit
            self._graphs[key] = g
        return g

    def _groups_fit(self) -> bool:
        """The running rows stay within the grouped decode kernels' window by the end of
        their decode (LLMEngine.groups_fit)."""
        return self.eng.groups_fit([len(r.prompt) + r.params.max_new_tokens for r in self.running])

    # ------------------------------------------------------------------ KV on demand
    def _grow_tables(self) -> None:
        """Before a step: every running request gets the block its write position enters
        (one block at a time); if the pool is out, preempt the youngest request and retry."""
        if not self.preempt or not self.running:
            return
        eng, BS = self.eng, self.eng.block_size
        while True:
            short = [r for r in self.running if r.pos // BS >= len(r.blocks)]
            if not short:
                return
            grown, failed = [], False
            for r in short:
                try:
                    b = eng._retry(lambda: eng.kv.allocator.alloc(1))[0]
                except MemoryError:
                    failed = True
                    break
                r.blocks.append(b)
                grown.append((self.running.index(r), len(r.blocks) - 1, b))
            if grown:
                idx = torch.tensor(grown, dtype=torch.long)
                m = self._master
                m.block_tables[idx[:, 0].to(m.block_tables.device), idx[:, 1].to(m.block_tables.device)] = \
                    idx[:, 2].to(device=m.block_tables.device, dtype=torch.int32)
            if not failed:
                return
            self._preempt_youngest()

    def _preempt_youngest(self) -> None:
        """Free the most recently admitted running request's blocks and re-queue it at the
        front of the waiting queue with its generated tokens appended to its prompt."""
        if self._pending is not None:       # every issued step's tokens reach the host first
            p, self._pending = self._pending, None
            self._process(p)
        if self.prefilling:
            # mixed steps: prompts being chunk-prefilled hold their whole prompt's blocks and
            # have produced no token yet -- re-queue the latest of them first (the
            # last running row used to fail while prefilling prompts held the blocks it needed)
            v = max(self.prefilling, key=lambda r: (r.t_arrival, r.rid))
            self.eng.kv.allocator.free(v.blocks)
            v.blocks, v.res, v.cached, v.filled = [], None, 0, 0
            self.prefilling = [r for r in self.prefilling if r is not v]
            v.preemptions += 1
            self.preempted += 1
            with self._cv:
                self.waiting.appendleft(v)
            return
        if not self.running:
            return
        v = max(self.running, key=lambda r: (r.t_arrival, r.rid))   # the latest arrival
        if len(self.running) == 1 and v.pos // self.eng.block_size >= len(v.blocks):
            # alone and still out of blocks: it can never finish in this pool
            self.eng.kv.allocator.free(v.blocks)
            v.blocks = []
            v.done = True
            if not v.future.done():
                v.future.set_exception(MemoryError("KV cache exhausted by a single request"))
            self._compact([])
            self._update_shared()
            return
        self.eng.kv.allocator.free(v.blocks)
        v.blocks, v.res, v.cached = [], None, 0
        keep = [i for i, r in enumerate(self.running) if r is not v]
        self._compact(keep)
        v.prompt = v.prompt[:v.orig_len] + list(v.out)
        v.gen_base = len(v.out)
        v.preemptions += 1
        self.preempted += 1
        with self._cv:
            self.waiting.appendleft(v)
        self._update_shared()

    def _decode(self) -> None:
        eng = self.eng
        self._grow_tables()
        n = len(self.running)
        if n == 0:
            return
        bp = _bucket(n, eng.max_batch) if self.pad_buckets else n
        greedy = all(r.params.temperature <= 0 for r in self.running)
        fit = self._groups_fit()
        grouped = self._nshared > 0 or eng.group_without_prefix(n, fit)
        g = self._graph(bp, greedy, grouped, fit)
        if eng.lpt:
            # re-rank only when the running set changed (admission / retirement)
            eng.set_order(g, [len(r.prompt) + len(r.out) for r in self.running], key=self._version)
        if grouped and g.groups_fit:
            eng.set_groups(g, [r.blocks for r in self.running],
                           [len(r.prompt) + r.params.max_new_tokens for r in self.running], self._nshared,
                           key=(self._version, self._nshared), ids=[r.rid for r in self.running])
        t0 = time.perf_counter()
        with tracing.span("sched.decode", running=n, bucket=bp, cascade=self._nshared > 0):
            if eng.use_graphs:
                if g.graph is None:
                    if self._pool is None:
                        self._pool = torch.cuda.graph_pool_handle()
                    eng._capture(g, self._pool)
                g.graph.replay()
            else:
                eng._step_body(g)
        eng.stats.generated_tokens += n
        self.steps += 1
        for r in self.running:
            r.pos += 1
        snap = list(self.running)
        if g.out.device.type == "cuda" or self.lag_cpu:
            if g.out.device.type == "cuda":
                if self._host is None:
                    self._host = [torch.empty(eng.max_batch, dtype=torch.long, pin_memory=True) for _ in range(2)]
                host = self._host[self._flip]
                self._flip ^= 1
                host[:n].copy_(g.out[:n], non_blocking=True)
                err = comm.collective_error_snapshot()
                ev = torch.cuda.Event()
                ev.record()
            else:
                host, err, ev = g.out[:n].clone(), comm.collective_error_snapshot(), None
            prev, self._pending = self._pending, (ev, host, snap, err)
            if prev is not None:
                self._process(prev)          # step t-1's tokens while step t runs
        else:
            self._process((None, g.out[:n].clone(), snap, comm.collective_error_snapshot()))
        eng.stats.decode_s += time.perf_counter() - t0

    def _process(self, pending) -> None:
        # a readback taken out of ``_pending`` stays reachable while it is processed: if it
        # raises (a collective-error snapshot, register_prefixes, _place), _fail_all still
        # frees the KV blocks and resolves the futures of a mixed step's completing prompts,
        # which are in neither ``running`` nor ``prefilling`` yet
        self._processing = pending
        self._process_one(pending)
        self._processing = None

    def _process_one(self, pending) -> None:
        if isinstance(pending[0], str):      # ("mixed", ...): a mixed step's readback
            self._process_mixed(pending)
            return
        ev, host, snap, err = pending
        if ev is not None:
            ev.synchronize()
        comm.raise_on_collective_error(err)
        toks = host[:len(snap)].tolist()
        finished = []
        for r, t in zip(snap, toks):
            if r.done:
                continue                      # the extra lagged step of a finished request
            self._emit(r, t)
            if self._finished(r):
                r.done = True
                finished.append(r)
        if finished:
            for r in finished:
                self._retire(r)
            keep = [i for i, r in enumerate(self.running) if not r.done]
            self._compact(keep)
            self._update_shared()

    def _emit(self, r: Request, tok: int) -> None:
        r.out.append(int(tok))
        self.generated += 1
        if r.on_token is not None:
            try:
                r.on_token(r.rid, int(tok))
            except Exception:  # noqa: BLE001 - a client callback must not stop the engine
                r.on_token = None

    def _finished(self, r: Request) -> bool:
        if len(r.out) >= r.params.max_new_tokens:
            return True
        return r.params.stop_on_eos and r.out[-1] == self.eng.cfg.eos_token_id

    def _retire(self, r: Request) -> None:
        self.completed += 1
        self.completed_short += len(r.out) < r.params.max_new_tokens
        self.eng.kv.allocator.free(r.blocks)
        r.blocks = []
        if not r.future.done():
            r.future.set_result(list(r.out))

    def _compact(self, keep: list[int]) -> None:
        """Move the surviving slots to [0, len(keep)) (one row gather per state tensor)."""
        m, n, k = self._master, len(self.running), len(keep)
        if keep != list(range(k)):
            idx = torch.tensor(keep, dtype=torch.long, device=m.tokens.device)
            for name in ("tokens", "positions", "context_lens", "valid", "block_tables", "inv_temp",
                         "top_k", "top_p"):
                t = getattr(m, name)
                t[:k] = t[idx]
        m.valid[k:n].zero_()
        m.context_lens[k:n].zero_()
        m.positions[k:n].zero_()
        m.tokens[k:n].zero_()
        self.running = [self.running[i] for i in keep]
        self._version += 1

    def _update_shared(self) -> None:
        """Cascade decode applies when all running slots share leading cached blocks."""
        rs = self.running
        ns = self.eng._shared_prefix_blocks([r.blocks for r in rs], [r.cached for r in rs]) if rs else 0
        if ns != self._nshared or (ns and self._shared_head != rs[0].blocks[:ns]):
            m = self._master
            if ns:
                st = torch.zeros(self.eng.max_blocks_per_seq, dtype=torch.int32)
                st[:ns] = torch.tensor(rs[0].blocks[:ns], dtype=torch.int32)
                m.shared_table.copy_(st.to(m.shared_table.device))
            m.shared_len.fill_(ns * self.eng.block_size)
            self._nshared = ns
            self._shared_head = rs[0].blocks[:ns] if ns else []
