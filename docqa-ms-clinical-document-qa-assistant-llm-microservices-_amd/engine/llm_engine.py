"""Generation engine for the llm-qa service: batched varlen prefill + HIP-graph decode.

One decode step for a batch bucket is captured once into a HIP graph (torch.cuda.graph
on ROCm) that contains the whole step: slot computation from the block table, the 32/80
layer forward, greedy/top-k/top-p sampling and the in-place advance of the step state
(positions, context lengths, next input token).  The host therefore only enqueues
``graph.replay()`` per token -- no per-layer launches, no host<->device syncs inside the
decode loop (a Llama-3-8B step is ~230 kernels; eager launch overhead would otherwise
dominate at small batch: MI355X_MICROARCH.md "graph-replay-floor").

Prefill packs all prompts of a batch into one varlen token stream (cu_seqlens), split
into sub-batches of at most ``max_prefill_tokens`` tokens; only the last position of
each prompt is projected through the LM head.

Reference parity: this is what ``RetrievalQA.invoke`` -> ``ChatOllama`` does per
request in the reference (llm-qa/main.py:117, one request at a time, greedy at T=0).
"""
from __future__ import annotations

import json
import itertools
import os
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import ops
from ..parallel import comm
from ..utils import tracing
from ..models.llama import AttnMeta, LlamaModel
from .kv_cache import KVCache, TailCache, chain_keys

_PREFILL_LOG = os.environ.get("DOCQA_PREFILL_LOG") == "1"   # one JSON line per prefill chunk
_PREFILL_DUMP = os.environ.get("DOCQA_PREFILL_DUMP", "")       # dir: save paged-prefill shapes for replay
# dir: save one cascade decode batch's tables / lengths / group plan for kernel replay
# (scripts/decode_replay_probe.py); the first DOCQA_DECODE_DUMP_SKIP batches are skipped
_DECODE_DUMP = os.environ.get("DOCQA_DECODE_DUMP", "")
_DECODE_DUMP_SKIP = [int(os.environ.get("DOCQA_DECODE_DUMP_SKIP", "1"))]


@dataclass
class SamplingParams:
    max_new_tokens: int = 128
    temperature: float = 0.0      # 0 -> greedy (the reference's ChatOllama temperature=0)
    top_k: int = 0
    top_p: float = 1.0
    stop_on_eos: bool = True
    seed: int = 0


@dataclass
class Reservation:
    """KV blocks reserved for a batch (LLMEngine.reserve): per prompt its block table and
    the number of leading tokens already in the prefix cache; ``copies``: token-granular
    prefix hits (source block, destination block, rows) to copy before the prefill, their
    source blocks pinned until then."""
    tables: list
    cached: list
    max_new_tokens: int
    n: int
    copies: list = field(default_factory=list)
    keys: list | None = None   # per prompt: chained block keys (kv_cache.chain_keys)


@dataclass
class Launched:
    """A batch enqueued by LLMEngine.launch: its reservation, the pinned host buffer its
    tokens are copied to and the (prefill start, prefill end, decode end) events."""
    reservation: Reservation
    host: torch.Tensor
    events: list | None
    params: "SamplingParams"
    t0: float
    t1: float
    # pinned copy of the TP all-reduce's error word behind the batch's kernels (None at TP 1)
    ar_err: torch.Tensor | None = None

    @property
    def done_event(self):
        return self.events[2] if self.events else None

    @property
    def start_event(self):
        return self.events[0] if self.events else None


@dataclass
class GenStats:
    prefill_s: float = 0.0
    decode_s: float = 0.0
    prompt_tokens: int = 0
    generated_tokens: int = 0
    cached_tokens: int = 0     # prompt tokens served from the prefix cache
    # distinct KV blocks one decode step's attention reads at its first step (the cascade
    # prefix counted once) -- the HBM floor of decode attention, summed over batches
    attn_kv_blocks: int = 0
    attn_batches: int = 0


def _bucket(n: int, cap: int) -> int:
    b = 1
    while b < n:
        b *= 2
    return min(b, cap)


def _prefill_inputs(prompts: list[list[int]], tables: list[list[int]], cached: list[int], BS: int):
    """Packed prefill inputs of the uncached prompt tails, vectorised (the per-token Python
    loop cost ~12 ms for a 256-prompt batch, with the GPU idle): token ids, positions,
    paged-cache slots and cu_seqlens, int32 numpy arrays."""
    new = np.array([len(p) - c for p, c in zip(prompts, cached)], dtype=np.int64)
    total = int(new.sum())
    ids = np.fromiter(itertools.chain.from_iterable(p[c:] for p, c in zip(prompts, cached)),
                      dtype=np.int32, count=total)
    cu = np.zeros(len(prompts) + 1, dtype=np.int32)
    np.cumsum(new, out=cu[1:])
    rows = np.repeat(np.arange(len(prompts)), new)
    pos = np.arange(total, dtype=np.int64) - cu[:-1].astype(np.int64)[rows] + np.asarray(cached, np.int64)[rows]
    tbm = np.zeros((len(tables), max(len(t) for t in tables)), dtype=np.int64)
    for r, t in enumerate(tables):
        tbm[r, :len(t)] = t
    slots = tbm[rows, pos // BS] * BS + pos % BS
    return ids, pos.astype(np.int32), slots.astype(np.int32), cu


def _upload(dst: torch.Tensor, src: torch.Tensor) -> None:
    """Host -> device copy that never blocks the host: from pinned memory, stream-ordered.
    (A copy from pageable memory waits for the stream -- after a prefill launch, for the
    whole prefill -- and the decode set-up that follows would then run with the GPU idle.)"""
    if dst.device.type == "cuda":
        dst.copy_(src.pin_memory(), non_blocking=True)
    else:
        dst.copy_(src)


_GROUP_NOPREFIX = os.environ.get("DOCQA_GROUP_NOPREFIX", "1") == "1"
_GROUP_NOPREFIX_MIN = int(os.environ.get("DOCQA_GROUP_NOPREFIX_MIN_BATCH", "32"))


def _split_groups_on() -> bool:
    return os.environ.get("DOCQA_GROUP_SPLIT", "1") == "1"


def _persist_groups_on() -> bool:
    """Persistent grouped decode (bins of work items per workgroup) on top of the split
    plan, DOCQA_GROUP_PERSIST=1.  Off by default: one workgroup per item measured 5 %
    faster end to end (153.4 vs 145.9 q/s, decode 1146 vs 1230 ms per batch, same box;
    profiles/r3_ab_group_persist.log)."""
    return _split_groups_on() and os.environ.get("DOCQA_GROUP_PERSIST", "0") == "1"


def _inline_prefix_on() -> bool:
    """Split plans whose items start at block 0: every group attends the shared cascade prefix
    itself (L2 hits after the first group) instead of a separate prefix kernel + merge --
    decode 1113-1116 vs 1140-1150 ms per 256-question batch (profiles/r4_inline_prefix_ab.log)."""
    return _split_groups_on() and os.environ.get("DOCQA_GROUP_INLINE_PREFIX", "1") == "1"


def _group_wave_on() -> bool:
    """Split plans run on the wave-parallel grouped decode kernel (attn_decode.hip
    paged_decode_group_wave_kernel, DOCQA_GROUP_WAVE=1..4, default 1; 0 = the cooperative
    kernel).  Its best plan has fewer, longer items: 66-82 items per KV head at batch 256
    run 69.6-69.8 us against 73.3 us at the cooperative kernel's 132
    (profiles/r5_group_wave_variants.log)."""
    return os.environ.get("DOCQA_GROUP_WAVE", "1") != "0"


def _defer_groups_on() -> bool:
    """Split plan with every group merged by the merge kernel (ops.split_decode_groups
    defer=True): the cascade-prefix kernel then runs on a side stream beside the group
    kernel (AttnMeta.decode_defer)."""
    return _split_groups_on() and os.environ.get("DOCQA_GROUP_DEFER", "0") == "1"


def _identity_groups(bp: int, dev, hkv: int = 8) -> torch.Tensor:
    cap = (bp + 1) // 2
    if _split_groups_on():
        # split plan [2, bp, 8] (persistent: [3, bp, 8]): consecutive unsplit quads until
        # set_groups runs
        persist = _persist_groups_on()
        # persistent / deferred plans: every quad writes a partial that the merge kernel
        # folds with the prefix (nothing may read the forked prefix kernel's partials)
        all_partial = persist or _defer_groups_on()
        # plan rows (work items): DOCQA_GROUP_CAP_MULT x the bucket; a plan that does not fit
        # doubles its tiles per item (ops.split_decode_groups)
        rows = max(bp, 1) * max(1, int(os.environ.get("DOCQA_GROUP_CAP_MULT", "1")))
        g = torch.full((3 if persist else 2, rows, 8), -1, dtype=torch.int32)
        g[:2, :, 4:] = 0
        g[0, :, 6] = -1
        nq = (bp + 3) // 4
        for i in range(nq):
            q = list(range(4 * i, min(4 * i + 4, bp)))
            g[0, i, :len(q)] = torch.tensor(q, dtype=torch.int32)
            g[0, i, 5] = 1 << 20
            if all_partial:
                g[0, i, 4] = 0
                g[0, i, 6] = i
                g[0, i, 7] = i          # merge row of the item (last-arriver merge)
                g[1, i, :len(q)] = torch.tensor(q, dtype=torch.int32)
                g[1, i, 4], g[1, i, 5] = i, 1
            else:
                g[0, i, 6] = -1
        if persist:   # one quad per bin (persist_bins >= bp / 4)
            nb = ops.persist_bins(max(bp, 1), hkv)
            for i in range(nq):
                g[2, i % nb, i // nb] = i
        return g.to(dev)
    g = torch.full((cap * 4,), -1, dtype=torch.int32)
    g[:bp] = torch.arange(bp, dtype=torch.int32)   # consecutive quads until set_groups runs
    return g.to(dev)


class _DecodeGraph:
    """Static buffers + captured graph for one batch bucket."""

    def __init__(self, eng: "LLMEngine", bp: int):
        dev = eng.device
        self.bp = bp
        self.tokens = torch.zeros(bp, dtype=torch.int32, device=dev)
        self.positions = torch.zeros(bp, dtype=torch.int32, device=dev)
        self.context_lens = torch.zeros(bp, dtype=torch.int32, device=dev)
        self.valid = torch.zeros(bp, dtype=torch.int32, device=dev)
        self.block_tables = torch.zeros(bp, eng.max_blocks_per_seq, dtype=torch.int32, device=dev)
        self.inv_temp = torch.ones(bp, dtype=torch.float32, device=dev)
        self.top_k = torch.zeros(bp, dtype=torch.int32, device=dev)
        self.top_p = torch.ones(bp, dtype=torch.float32, device=dev)
        self.out = torch.zeros(bp, dtype=torch.long, device=dev)
        # cascade decode: block ids / length of the prompt prefix every row shares
        self.shared_table = torch.zeros(eng.max_blocks_per_seq, dtype=torch.int32, device=dev)
        self.shared_len = torch.zeros(1, dtype=torch.int32, device=dev)
        # decode-attention dispatch order (LPT: longest context first), a permutation of
        # [0, bp) per bucket -- never a view of another bucket's buffer
        self.order = torch.arange(bp, dtype=torch.int32, device=dev)
        self.order_key = None
        # grouped cascade decode: rows packed into groups of <= 4 by shared prefix-cache
        # blocks (room for bp / 2 groups; unused groups are all -1 and exit at once)
        self.groups = _identity_groups(bp, dev, eng.model.hkv)
        self.groups_key = None
        self.cascade = False
        self.greedy = True
        self.graph = None
        self.hkv = eng.model.hkv
        # the rows this graph serves reach <= ops.GROUP_MAX_BLOCKS blocks (the grouped decode
        # kernels' window): always true when the block table itself is that narrow
        self.groups_fit = eng.max_blocks_per_seq <= ops.GROUP_MAX_BLOCKS

    @classmethod
    def view_of(cls, master: "_DecodeGraph", bp: int) -> "_DecodeGraph":
        """Buffers for bucket ``bp`` that are the first ``bp`` slots of ``master``: graphs
        of every bucket then read/write ONE slot state, so a continuous-batching scheduler
        can change bucket between steps without copying state."""
        g = cls.__new__(cls)
        g.bp = bp
        for name in ("tokens", "positions", "context_lens", "valid", "block_tables", "inv_temp",
                     "top_k", "top_p", "out"):
            setattr(g, name, getattr(master, name)[:bp])
        g.shared_table, g.shared_len = master.shared_table, master.shared_len
        g.order = torch.arange(bp, dtype=torch.int32, device=master.tokens.device)
        g.order_key = None
        g.groups = _identity_groups(bp, master.tokens.device, master.hkv)
        g.groups_key = None
        g.cascade, g.greedy, g.graph = False, True, None
        g.groups_fit = master.groups_fit
        g.hkv = master.hkv
        return g


class LLMEngine:
    def __init__(self, model: LlamaModel, max_batch: int = 64, max_context: int = 2048,
                 block_size: int = 64, num_blocks: int | None = None, use_graphs: bool = True,
                 max_prefill_tokens: int = 65536, prefix_cache: bool = True,
                 kv_mem_fraction: float | None = None):
        """``num_blocks``: KV pool size; default ``max_batch`` full-context sequences, or --
        with ``kv_mem_fraction`` (env DOCQA_KV_MEM_FRACTION) on a GPU -- that fraction of the
        HBM still free after the weights, minus the prefill activation headroom (the block
        prefix cache keeps every block the running batches do not need)."""
        self.model = model
        self.cfg = model.cfg
        self.device = model.device
        self.max_batch = max_batch
        self.block_size = block_size
        self.max_blocks_per_seq = (max_context + block_size - 1) // block_size
        self.max_context = self.max_blocks_per_seq * block_size
        sw = getattr(model.cfg, "sliding_window", None)
        if sw is not None and self.max_context > sw:
            raise ValueError(f"max_context {self.max_context} exceeds the model's sliding window {sw}: "
                             "the attention kernels attend to the whole context")
        if getattr(model, "tp", 1) > 1:
            # TP prefill all-reduces ([tokens, hidden] bf16) stay inside the IPC all-reduce's
            # staging area (two-shot over all xGMI links) instead of falling back to RCCL
            from ..parallel import comm
            car = comm.custom_all_reduce()
            if car is not None:
                cap = car.max_elems // model.cfg.hidden // block_size * block_size
                max_prefill_tokens = max(block_size, min(max_prefill_tokens, cap))
        self.max_prefill_tokens = max_prefill_tokens
        if num_blocks is None:
            num_blocks = max_batch * self.max_blocks_per_seq + 1
            if kv_mem_fraction is None and os.environ.get("DOCQA_KV_MEM_FRACTION"):
                kv_mem_fraction = float(os.environ["DOCQA_KV_MEM_FRACTION"])
            if kv_mem_fraction and self.device.type == "cuda":
                # the HBM budget decides; when even max_batch full contexts do not fit beside the
                # weights (Llama-3-70B at batch 256: 8193 blocks = 164 GB next to 141 GB) the pool
                # is the budget: blocks are reserved per actual prompt + generation, admission
                # waits / the scheduler preempts when it runs out -- it must hold at least one
                # full-context sequence
                fb = self._blocks_from_free_memory(model, block_size, kv_mem_fraction)
                if num_blocks <= self._blocks_from_free_memory(model, block_size, 0.95):
                    num_blocks = max(num_blocks, fb)       # the full-context pool fits: never less
                elif fb >= self.max_blocks_per_seq + 1:
                    num_blocks = fb
                else:
                    raise MemoryError(f"KV pool: {fb} blocks fit in {kv_mem_fraction:.2f} of the free HBM, "
                                      f"one {self.max_context}-token sequence needs {self.max_blocks_per_seq + 1}")
        num_blocks = self._agree_across_tp(model, num_blocks)
        self.kv = KVCache(self.cfg.layers, num_blocks, model.hkv, self.cfg.head_dim, block_size,
                          self.device, model.dtype)
        self.use_graphs = use_graphs and self.device.type == "cuda"
        # TunableOp search for the decode buckets' library GEMMs (only the LM head below the
        # mid-M rows is left on hipBLASLt): off by default -- ~28 s of service start-up for no
        # measurable step time (docs/CONFIG.md)
        self.tune_decode_gemms = os.environ.get("DOCQA_TUNE_DECODE", "0") == "1"
        # reuse KV blocks of shared prompt prefixes (the fixed RAG instruction template)
        self.prefix_cache = prefix_cache and os.environ.get("DOCQA_PREFIX_CACHE", "1") == "1"
        # cascade decode attention (csrc/include/docqa_cascade.h): when every sequence of a
        # batch starts with the same cached prompt-prefix blocks (the RAG instruction
        # template), that prefix is attended once per step for the whole batch
        self.cascade = os.environ.get("DOCQA_CASCADE", "1") == "1"
        self.cascade_min_tokens = int(os.environ.get("DOCQA_CASCADE_MIN_TOKENS", "128"))
        self.cascade_min_batch = int(os.environ.get("DOCQA_CASCADE_MIN_BATCH", "4"))
        # LPT dispatch of the decode-attention workgroups (mixed context lengths cost ~15 %
        # in random order, benchmarks/bench_decode_attn.py MIX=random vs sorted)
        self.lpt = os.environ.get("DOCQA_DECODE_LPT", "1") == "1"
        # grouped cascade decode: rows sharing prefix-cache blocks attended together
        self.group_decode = os.environ.get("DOCQA_DECODE_GROUP", "1") == "1"
        # the prefix cache needs the native block manager (batched hash-keyed lookups)
        self._use_pc = self.prefix_cache and hasattr(self.kv.allocator, "match_alloc_batch")
        # token-granular prefix reuse below the block size (engine/kv_cache.py TailCache)
        # (each entry pins one block: at most an eighth of the pool)
        # 4096 (capped at an eighth of the pool): 0.766 -> 0.777 of prompt tokens cached at the
        # bench's batch 256, +0.8-1.6 % q/s same box vs 1024 (profiles/r4_knobs_items_tail.log)
        cap = min(int(os.environ.get("DOCQA_TAIL_CACHE", "4096")), num_blocks // 8)
        self.tail = TailCache(self.kv.allocator, block_size, cap) if self._use_pc and cap > 0 else None
        self._graphs: dict[tuple, _DecodeGraph] = {}
        self._pool = None
        self.stats = GenStats()

    @staticmethod
    def _agree_across_tp(model, num_blocks: int) -> int:
        """Every rank of a TP group must run the same block allocator (lockstep serving,
        identical preemption / eviction decisions): the smallest pool of the group."""
        import torch.distributed as dist

        from ..parallel import comm

        st = comm.state()
        if getattr(model, "tp", 1) > 1 and st.tp_size > 1 and dist.is_initialized():
            t = torch.tensor([num_blocks], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=st.tp_cpu_group or st.tp_group)
            num_blocks = int(t.item())
        return num_blocks

    def _blocks_from_free_memory(self, model, block_size: int, fraction: float) -> int:
        cfg = model.cfg
        free, _ = torch.cuda.mem_get_info(self.device)
        el = torch.finfo(model.dtype).bits // 8
        block_bytes = cfg.layers * 2 * model.hkv * block_size * cfg.head_dim * el
        # prefill activations at the token budget (hidden-sized buffers, QKV, the gate|up
        # product / SwiGLU output) twice over, + 6 GB for graph pools, workspaces and the index
        per_tok = (6 * cfg.hidden + (model.hq + 2 * model.hkv) * cfg.head_dim + 3 * model.inter) * el
        headroom = 2 * self.max_prefill_tokens * per_tok + (6 << 30)
        budget = int(free * fraction) - headroom
        return max(0, budget // block_bytes)

    # ------------------------------------------------------------------ prefill
    def _prefill(self, prompts: list[list[int]], tables: list[list[int]],
                 cached: list[int] | None = None, greedy: bool = False) -> torch.Tensor:
        """Prefill prompt tokens [cached[i], len) of each prompt (the first cached[i]
        tokens are prefix-cache hits already in the paged KV cache).  Returns the last
        position's logits per prompt, or (``greedy``) its greedy token id (the LM head's
        argmax fused into its GEMM: no [B, vocab] logits)."""
        dev, BS = self.device, self.block_size
        cached = list(cached or [0] * len(prompts))
        # chunked prefill: a prompt longer than the token budget is fed in budget-sized
        # pieces; each piece attends to the earlier ones through the paged cache (the
        # prefix-cache attention path), so activation memory stays bounded for the long
        # multi-patient synthese prompts
        budget = max(BS, self.max_prefill_tokens // BS * BS)
        for k, (p, tb) in enumerate(zip(prompts, tables)):
            while len(p) - cached[k] > budget:
                end = cached[k] + budget
                self._prefill([p[:end]], [tb], [cached[k]])
                cached[k] = end
        firsts = []
        i = 0
        while i < len(prompts):
            j, tok = i, 0
            while j < len(prompts) and (j == i or tok + len(prompts[j]) - cached[j] <= self.max_prefill_tokens):
                tok += len(prompts[j]) - cached[j]
                j += 1
            ids, pos, slots, cu = _prefill_inputs(prompts[i:j], tables[i:j], cached[i:j], BS)
            t_ids = torch.from_numpy(ids).to(dev, non_blocking=True)
            meta = AttnMeta(
                prefill=True,
                positions=torch.from_numpy(pos).to(dev, non_blocking=True),
                slot_mapping=torch.from_numpy(slots).to(dev, non_blocking=True),
                cu_seqlens=torch.from_numpy(cu).to(dev, non_blocking=True),
                max_len=max(len(p) - c for p, c in zip(prompts[i:j], cached[i:j])))
            if any(cached[i:j]):
                maxb = max(len(tb) for tb in tables[i:j])
                bt = torch.zeros(j - i, maxb, dtype=torch.int32)
                for r, tb in enumerate(tables[i:j]):
                    bt[r, :len(tb)] = torch.tensor(tb, dtype=torch.int32)
                meta.block_tables = bt.to(dev, non_blocking=True)
                meta.prefix_lens = torch.tensor(cached[i:j], dtype=torch.int32).to(dev, non_blocking=True)
            last = torch.from_numpy(cu[1:].astype(np.int64) - 1).to(dev, non_blocking=True)
            if _PREFILL_DUMP and meta.block_tables is not None:
                os.makedirs(_PREFILL_DUMP, exist_ok=True)
                torch.save({"cu": torch.tensor(cu, dtype=torch.int32), "ctx": torch.tensor(cached[i:j], dtype=torch.int32),
                            "bt": meta.block_tables.cpu()},
                           os.path.join(_PREFILL_DUMP, f"prefill_{time.time_ns()}.pt"))
            if _PREFILL_LOG:
                new = [len(p) - c for p, c in zip(prompts[i:j], cached[i:j])]
                print(json.dumps({"prefill_chunk": j - i, "new_sum": sum(new), "new_max": max(new),
                                  "cached_mean": sum(cached[i:j]) / (j - i), "cached_max": max(cached[i:j]),
                                  "cached_min": min(cached[i:j])}), flush=True)
            firsts.append(self.model.forward(t_ids, meta, self.kv.caches, logits_index=last, greedy_ids=greedy))
            i = j
        return torch.cat(firsts, 0)

    # ------------------------------------------------------------------ decode step
    def _step_body(self, g: _DecodeGraph) -> None:
        meta = self._decode_meta(g)
        if g.greedy:
            # greedy: the LM head's argmax is fused into its GEMM (no [B, vocab] logits)
            nxt = self.model.forward(g.tokens, meta, self.kv.caches, greedy_ids=True)
        else:
            nxt = self._select(self.model.forward(g.tokens, meta, self.kv.caches), g)
        ops.decode_advance(nxt.long().contiguous(), g.out, g.tokens, g.positions, g.context_lens, g.valid)

    def _decode_meta(self, g: _DecodeGraph) -> AttnMeta:
        """Attention metadata of one decode step of bucket ``g`` (slots of the new tokens,
        cascade prefix and row groups when the step attends a shared prefix)."""
        slots = ops.decode_slots(g.block_tables, g.positions, g.valid, self.block_size)
        meta = AttnMeta(prefill=False, positions=g.positions, slot_mapping=slots,
                        block_tables=g.block_tables, context_lens=g.context_lens,
                        max_context=self.max_context, seq_order=g.order if self.lpt else None)
        if g.cascade:
            meta.shared_table, meta.shared_len = g.shared_table, g.shared_len
            meta.cascade_chunks = self._cascade_chunks(g.bp)
            if self.group_decode and g.groups_fit and ops.grouped_decode_ok(
                    self.kv.caches[0][0], g.block_tables, self.model.hq, max_blocks=ops.GROUP_MAX_BLOCKS):
                meta.decode_groups = g.groups
                meta.decode_defer = g.groups.dim() == 3 and _defer_groups_on()
                meta.decode_inline = (g.groups.dim() == 3 and g.groups.shape[0] == 2 and _inline_prefix_on()
                                      and not _defer_groups_on())
        return meta

    def _select(self, logits, g: _DecodeGraph):
        from .. import ops

        if g.greedy:
            return self.model.greedy(logits)
        full = self.model.full_logits(logits).float()
        u = torch.rand(full.shape[0], device=full.device)
        return ops.sample(full, g.inv_temp, g.top_k, g.top_p, u)

    def _get_graph(self, bp: int, greedy: bool, cascade: bool = False, fit: bool = True) -> _DecodeGraph:
        fit = fit or self.max_blocks_per_seq <= ops.GROUP_MAX_BLOCKS
        key = (bp, greedy, cascade, fit)
        g = self._graphs.get(key)
        if g is None:
            g = _DecodeGraph(self, bp)
            g.greedy = greedy
            g.cascade = cascade
            g.groups_fit = fit
            self._graphs[key] = g
        return g

    def groups_fit(self, end_lens: list[int]) -> bool:
        """Whether every row of a decode batch -- at ``end_lens`` tokens by the end of its
        decode -- stays within the grouped decode kernels' window (ops.GROUP_MAX_BLOCKS
        blocks, 4096 tokens).  The block table is sized for MAX_CONTEXT (8192 in the llm-qa
        service: 128 blocks), but RAG prompts of ~1k tokens fit, so they take the grouped
        kernels (~70 us per layer at batch 256) instead of the per-row ring kernel (~160)."""
        if self.max_blocks_per_seq <= ops.GROUP_MAX_BLOCKS:
            return True
        BS = self.block_size
        return all((n + BS - 1) // BS <= ops.GROUP_MAX_BLOCKS for n in end_lens)

    def set_order(self, g: _DecodeGraph, lens: list[int], key=None) -> None:
        """Dispatch order of bucket ``g``'s decode rows: active rows [0, len(lens)) by
        descending context length, then the padded rows.  Contexts all grow by one token a
        step, so the order stays valid until the batch composition changes (``key``: skip
        the upload when it is unchanged)."""
        if key is not None and g.order_key == key:
            return
        order = sorted(range(len(lens)), key=lambda i: -lens[i]) + list(range(len(lens), g.bp))
        _upload(g.order, torch.tensor(order, dtype=torch.int32))
        g.order_key = key

    def set_groups(self, g: _DecodeGraph, tables: list[list[int]], lens: list[int], skip: int,
                   key=None, ids: list | None = None) -> None:
        """Pack the active rows of bucket ``g`` into groups of <= 4 that share prefix-cache
        blocks beyond the ``skip`` cascade-prefix blocks (ops.pack_decode_groups); padded
        rows take no group.  Static while the batch composition is unchanged (``key``).

        ``ids`` (a request id per row): when the rows are a subset of the rows the current
        split plan was built for -- requests only RETIRED and the survivors were compacted
        -- the plan's row ids are remapped instead of re-planned (a retired row's columns
        go empty; an item whose rows all retired exits at once, and since every item of a
        group carries the same rows, no group's merge ticket is left half-drawn).  A full
        re-plan runs on any admission, or once a quarter of the planned rows is gone."""
        if not self.group_decode or (key is not None and g.groups_key == key):
            return
        skip_in = skip
        if (ids is not None and g.groups.dim() == 3 and getattr(g, "plan_ids", None) is not None
                and g.plan_skip == skip_in and len(ids) * 4 >= len(g.plan_ids) * 3):
            plan = ops.remap_plan_rows(g.plan_host, g.plan_ids, ids)
            if plan is not None:
                _upload(g.groups, plan)
                g.groups_key = key
                return
        if g.groups.dim() == 3:   # split plan: long groups over several workgroups
            cap = g.groups.shape[1]
            quads = ops.pack_decode_groups(tables, lens, skip, self.block_size, (g.bp + 1) // 2)
            if _inline_prefix_on() and not _defer_groups_on() and g.groups.shape[0] == 2:
                skip = 0   # the kernel attends the shared prefix inside each group
            bins = ops.persist_bins(cap, self.model.hkv) if g.groups.shape[0] == 3 else 0

            # the per-quad tile lists do not depend on the budget: computed once for every
            # budget the auto search tries (38 -> ~6 ms of host planning per 256-row replan)
            per_quad = [ops.group_tiles_by_position(tables, lens, list(qd), skip, self.block_size) for qd in quads]

            def split(tiles):
                return ops.split_decode_groups(quads, tables, lens, skip, self.block_size, cap, tiles,
                                               bins=bins, defer=_defer_groups_on(), per_quad=per_quad)

            tiles = os.environ.get("DOCQA_GROUP_TILES", "auto")
            if tiles == "auto":
                # the tiles-per-item budget whose plan has the most items, at most
                # DOCQA_GROUP_ITEMS per KV head: ~1.4 rounds of the chip's 96 workgroup slots per head.  At the bench's
                # batch 256 that is 40 tiles, ~130 items (12 -- which overflowed the plan into
                # 24-tile items, ~200 -- ran 1.5 % fewer q/s; 20-32 and 56 slower too:
                # profiles/r4_group_plan_tiles_sweep.log); smaller buckets keep smaller items,
                # so their few groups still fill the chip
                # (a budget whose plan overflows the rows comes back doubled, so take the plan
                # with the MOST items within the target rather than the first that fits:
                # batch 64 / 128 run best at 54 / 106 items, 12 tiles)
                target = int(os.environ.get("DOCQA_GROUP_ITEMS", "82" if _group_wave_on() else "132"))
                # items fall as the budget grows: the first budget within the target gives
                # the plan with the most items (the search stops there -- host time per
                # replan matters when serving retires rows every few steps)
                plan = None
                for budget in (8, 12, 16, 24, 32, 40, 48, 64, 96, 128):
                    p = split(budget)
                    if int((p[0, :, :4] >= 0).any(1).sum()) <= target:
                        plan = p
                        break
                if plan is None:
                    plan = split(128)
            else:
                plan = split(int(tiles))
            _upload(g.groups, plan)
            g.groups_key = key
            g.plan_ids = list(ids) if ids is not None else None
            g.plan_host, g.plan_skip = plan, skip_in
            if os.environ.get("DOCQA_GROUP_PLAN_LOG", "0") == "1":
                used = int((plan[0, :, :4] >= 0).any(1).sum())
                print(f"[group plan] bp {g.bp} groups {len(quads)} items {used} cap {cap}", flush=True)
            return
        cap = g.groups.numel() // 4
        quads = ops.pack_decode_groups(tables, lens, skip, self.block_size, cap)
        flat = torch.full((cap * 4,), -1, dtype=torch.int32)
        for i, qd in enumerate(quads):
            flat[4 * i:4 * i + len(qd)] = torch.tensor(qd, dtype=torch.int32)
        _upload(g.groups, flat)
        g.groups_key = key

    def group_without_prefix(self, B: int, fit: bool = True) -> bool:
        """The grouped split-plan decode with the prefix attended inline needs no prefix
        shared by EVERY row: its items start at block 0 and rows are grouped by whatever
        prefix-cache blocks they share (retrieved chunks).  So batches without a common
        template prefix -- the reference QA template puts the context first -- take the
        wave-parallel grouped kernel too instead of the per-row ring kernel (round 5: 162 us
        vs ~70 us per layer at batch 256, profiles/r5_head_kernel_stats.txt).
        DOCQA_GROUP_NOPREFIX=0 disables; from DOCQA_GROUP_NOPREFIX_MIN_BATCH rows (32).
        ``fit``: :meth:`groups_fit` of the batch's rows."""
        return (B >= _GROUP_NOPREFIX_MIN and _GROUP_NOPREFIX and self.group_decode and self.cascade and fit
                and self.device.type == "cuda" and _split_groups_on() and _inline_prefix_on()
                and not _defer_groups_on() and not _persist_groups_on()
                and ops.grouped_decode_ok(self.kv.caches[0][0], torch.empty(0, self.max_blocks_per_seq),
                                          self.model.hq, max_blocks=ops.GROUP_MAX_BLOCKS))

    def _cascade_chunks(self, bp: int) -> int:
        """Key chunks of the shared-prefix kernel: about 256 workgroups of (64 rows, KV
        head, chunk) in total, 1..16 chunks (DOCQA_CASCADE_CHUNKS overrides)."""
        env = int(os.environ.get("DOCQA_CASCADE_CHUNKS", "0"))
        if env > 0:
            return env
        tiles = (bp + 63) // 64 * self.model.hkv
        return max(1, min(16, 256 // max(1, tiles)))

    def _shared_prefix_blocks(self, tables: list[list[int]], cached: list[int]) -> int:
        """Number of leading prefix-cache blocks that are the SAME physical blocks in every
        row of the batch (0 if cascade decode does not apply)."""
        B, BS = len(tables), self.block_size
        if (not self.cascade or B < self.cascade_min_batch
                or not ops.cascade_ok(self.kv.caches[0][0], torch.empty(0, self.max_blocks_per_seq), self.model.hq)):
            return 0
        n = min(c // BS for c in cached)
        first = tables[0]
        k = 0
        while k < n and all(t[k] == first[k] for t in tables):
            k += 1
        return k if k * BS >= self.cascade_min_tokens else 0

    def _capture(self, g: _DecodeGraph, pool=None) -> None:
        """``pool``: graph memory pool handle (default: this engine's own); a scheduler
        that owns its graphs passes its own so their lifetimes stay independent."""
        # warm up on a side stream (allocator + hipBLASLt heuristics), then capture.
        # Decode GEMMs are skinny (M = batch bucket) and their shapes are fixed per bucket,
        # so they are worth an exhaustive hipBLASLt/rocBLAS solution search (PyTorch
        # TunableOp) during the eager warm-up; the winners are baked into the graph.
        # Prefill shapes vary per batch and keep the default heuristics.
        tune = self.tune_decode_gemms
        tunable = getattr(torch.cuda, "tunable", None)
        import logging
        import threading

        logging.getLogger("docqa.engine").info("decode graph capture: bucket %d cascade %s greedy %s (thread %s)",
                                               g.bp, getattr(g, "cascade", None), getattr(g, "greedy", None),
                                               threading.current_thread().name)
        if tune and tunable is not None:
            tunable.enable(True)
            tunable.tuning_enable(True)
            # time candidates on cold weights: a decode step streams every layer's weights
            # from HBM once (16 GB >> the 256 MB MALL), so solutions must be ranked with
            # the operands rotated past the caches, not re-read hot
            rot = int(os.environ.get("DOCQA_TUNE_ROTATE_MB", "512"))
            if rot > 0 and hasattr(tunable, "set_rotating_buffer_size"):
                tunable.set_rotating_buffer_size(rot)
        saved = [t.clone() for t in (g.tokens, g.positions, g.context_lens)]
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self._step_body(g)
            torch.cuda.current_stream().wait_stream(s)
            for t, v in zip((g.tokens, g.positions, g.context_lens), saved):
                t.copy_(v)
            if tune and tunable is not None:
                tunable.tuning_enable(False)
            graph = torch.cuda.CUDAGraph()
            if pool is None:
                if self._pool is None:
                    self._pool = torch.cuda.graph_pool_handle()
                pool = self._pool
            # thread_local: the serving front end keeps embedding / searching / syncing on
            # its prep thread while the scheduler thread captures a new bucket lazily; in the
            # default global mode any sync on ANY thread invalidates the capture (and fails
            # that thread's op: hipErrorStreamCaptureUnsupported)
            with torch.cuda.graph(graph, pool=pool, capture_error_mode="thread_local"):
                self._step_body(g)
        finally:
            if tune and tunable is not None:
                tunable.enable(False)
        for t, v in zip((g.tokens, g.positions, g.context_lens), saved):
            t.copy_(v)
        g.graph = graph

    @torch.inference_mode()
    def warm_graphs(self, batch: int, greedy: bool = True) -> None:
        """Capture the decode graphs (plain and cascade) of the bucket serving ``batch``
        sequences now, with empty slots (valid 0: nothing is written to the KV cache), so
        the first batch that hits the cascade path does not pay a capture / GEMM tuning."""
        if not self.use_graphs:
            return
        bp = _bucket(batch, self.max_batch)
        for cascade in ([False, True] if self.cascade else [False]):
            g = self._get_graph(bp, greedy, cascade)
            if g.graph is None:
                for t in (g.valid, g.positions, g.context_lens, g.tokens):
                    t.zero_()
                g.shared_len.zero_()
                self._capture(g)

    # ------------------------------------------------------------------ generate
    @torch.inference_mode()
    def generate(self, prompts: list[list[int]], params: SamplingParams | None = None,
                 on_step=None) -> list[list[int]]:
        """``on_step(step, total)`` is called from the host decode loop after each step is
        enqueued (the serving pipeline uses it to start the next batch's preparation a few
        steps before this one ends)."""
        params = params or SamplingParams()
        out: list[list[int]] = []
        for i in range(0, len(prompts), self.max_batch):
            out.extend(self._generate_batch(prompts[i:i + self.max_batch], params, on_step))
        return out

    def _generate_batch(self, prompts: list[list[int]], params: SamplingParams,
                        on_step=None) -> list[list[int]]:
        return self.collect(self.launch(prompts, params, on_step))

    def reserve(self, prompts: list[list[int]], params: SamplingParams,
                gen_tokens: int | None = None) -> "Reservation":
        """KV blocks of a batch: the longest cached prompt prefix of each prompt (prefix
        cache, refcounted) + fresh blocks for the rest of the prompt and the generation.
        Host-only work (~12 ms for 256 RAG prompts), so a pipelined caller runs it on its
        preparation thread while the previous batch decodes; pass the result to
        :meth:`launch` (or :meth:`release` it)."""
        lens = [len(p) for p in prompts]
        gen = params.max_new_tokens if gen_tokens is None else gen_tokens
        need = max(lens) + gen
        if need > self.max_context:
            raise ValueError(f"prompt+generation {need} exceeds max_context {self.max_context}")
        with tracing.span("engine.reserve", seqs=len(prompts)):
            return self._reserve(prompts, params, lens, gen)

    def _reserve(self, prompts, params, lens, gen: int | None = None) -> "Reservation":
        """``gen``: generated tokens to reserve blocks for (default: all max_new_tokens; the
        continuous scheduler reserves a block ahead and grows tables as decode goes)."""
        alloc = self.kv.allocator
        BS = self.block_size
        gen = params.max_new_tokens if gen is None else gen
        need = [self.kv.blocks_for(n + gen) for n in lens]
        r = Reservation([], [], params.max_new_tokens, len(prompts))
        if not self._use_pc:
            try:
                for n in need:
                    r.tables.append(self._retry(lambda n=n: alloc.alloc(n)))
            except BaseException:
                self.release(r)   # no partial reservation may outlive a failed one
                raise
            r.cached = [0] * len(prompts)
            return r
        # one native call for the batch: longest cached full-block prefix of every prompt
        # (chained keys computed here, reused by the token-granular cache and registration)
        r.keys = [chain_keys(p, BS, (len(p) + BS - 1) // BS) for p in prompts]
        hits, r.tables = self._retry(lambda: alloc.match_alloc_batch(
            [k[1:len(p) // BS + 1] for k, p in zip(r.keys, prompts)], lens, need))
        try:
            for i, p in enumerate(prompts):
                k, c = hits[i], hits[i] * BS
                if self.tail is not None and k < len(r.tables[i]):
                    t = self.tail.lookup(p, k, len(p) - 1 - c, keys=r.keys[i])
                    if t is not None:
                        r.copies.append((t[0], r.tables[i][k], t[1]))
                        c += t[1]
                r.cached.append(c)
        except BaseException:
            self.release(r)
            raise
        return r

    def _retry(self, fn):
        """``fn()``; on KV-pool exhaustion, once more after the blocks pinned by the
        token-granular prefix cache give way."""
        try:
            return fn()
        except MemoryError:
            if self.tail is None or not self.tail.shrink(max(1, len(self.tail))):
                raise
            return fn()

    def release(self, r: "Reservation") -> None:
        for tb in r.tables:
            self.kv.allocator.free(tb)
        r.tables = []
        if r.copies:
            self.tail.unpin([src for src, _, _ in r.copies])
            r.copies = []

    def queue_prefix_copies(self, r: "Reservation") -> None:
        """Queue the token-granular prefix hits' K/V row copies of a reservation (before its
        prefill reads them) and drop the pins on their sources (stream order keeps them
        valid until copied)."""
        if r.copies:
            self._copy_prefix_rows(r.copies)
            self.tail.unpin([src for src, _, _ in r.copies])
            r.copies = []

    def register_prefixes(self, prompts: list[list[int]], tables: list[list[int]], keys=None) -> None:
        """Publish prefilled prompts to the block prefix cache (full blocks, one native
        call) and to the token-granular cache (every block position)."""
        if not self._use_pc:
            return
        BS = self.block_size
        keys = [k if k is not None else chain_keys(p, BS, (len(p) + BS - 1) // BS)
                for p, k in zip(prompts, keys or [None] * len(prompts))]
        self.kv.allocator.register_batch([k[1:len(p) // BS + 1] for k, p in zip(keys, prompts)], tables)
        if self.tail is not None:
            for p, tb, k in zip(prompts, tables, keys):
                self.tail.register(p, tb, keys=k)

    def _copy_prefix_rows(self, copies: list) -> None:
        """K/V rows [0, m) of each source block -> the same rows of its destination block,
        every layer (token-granular prefix hits, queued before the prefill reads them)."""
        if self.device.type == "cuda" and getattr(self, "_cache_ptrs", None) is None:
            self._cache_ptrs = torch.tensor([t.data_ptr() for kv in self.kv.caches for t in kv],
                                            dtype=torch.int64, device=self.device)
        ops.kv_copy_rows(self.kv.caches, copies, getattr(self, "_cache_ptrs", None))

    def launch(self, prompts: list[list[int]], params: SamplingParams | None = None, on_step=None,
               reserved: "Reservation | None" = None) -> "Launched":
        """Enqueue one batch (<= max_batch prompts): prefill, first-token selection and every
        decode step (HIP-graph replays), then an async copy of the generated ids to pinned
        host memory -- WITHOUT waiting for any of it.  :meth:`collect` waits and returns the
        tokens.  Launching batch i+1 before collecting batch i queues its prefill right
        behind batch i's last decode step, so the host work between batches (collecting,
        detokenising, the next batch's set-up) never leaves the GPU idle.  Batches on one
        stream share the bucket's graph buffers; every write to them is stream-ordered."""
        with tracing.span("engine.launch", seqs=len(prompts)):
            return self._launch(prompts, params, on_step, reserved)

    def _launch(self, prompts, params, on_step, reserved) -> "Launched":
        params = params or SamplingParams()
        B = len(prompts)
        if B > self.max_batch:
            raise ValueError(f"launch: {B} prompts > max_batch {self.max_batch}")
        dev = self.device
        cuda = dev.type == "cuda"
        lens = [len(p) for p in prompts]
        if reserved is not None and (reserved.n != B or reserved.max_new_tokens != params.max_new_tokens):
            self.release(reserved)
            reserved = None
        r = reserved if reserved is not None else self.reserve(prompts, params)
        tables, cached = r.tables, r.cached
        alloc = self.kv.allocator
        use_pc = self._use_pc
        try:
            greedy = params.temperature <= 0.0
            t0 = time.perf_counter()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if cuda else None
            if cuda:
                ev[0].record()
            self.queue_prefix_copies(r)
            with tracing.span("engine.prefill", seqs=B, tokens=sum(lens) - sum(cached)):
                logits = self._prefill(prompts, tables, cached, greedy=greedy)
            if use_pc:
                with tracing.span("engine.register", seqs=B):
                    self.register_prefixes(prompts, tables, r.keys)
            self.stats.cached_tokens += sum(cached)
            nshared = self._shared_prefix_blocks(tables, cached)
            self.stats.attn_kv_blocks += nshared + len({b for t in tables for b in t[nshared:]})
            self.stats.attn_batches += 1
            fit = self.groups_fit([n + params.max_new_tokens for n in lens])
            grouped = nshared > 0 or self.group_without_prefix(B, fit)
            g = self._get_graph(_bucket(B, self.max_batch) if self.use_graphs else B, greedy, grouped, fit)
            if grouped:
                g.shared_len.fill_(0)
            if nshared:
                st = torch.zeros(self.max_blocks_per_seq, dtype=torch.int32)
                st[:nshared] = torch.tensor(tables[0][:nshared], dtype=torch.int32)
                _upload(g.shared_table, st)
                g.shared_len.fill_(nshared * self.block_size)
            # state for the first decode step
            bt = torch.zeros(g.bp, self.max_blocks_per_seq, dtype=torch.int32)
            for i, tb in enumerate(tables):
                bt[i, :len(tb)] = torch.tensor(tb, dtype=torch.int32)
            _upload(g.block_tables, bt)
            vl = torch.zeros(g.bp, dtype=torch.int32)
            vl[:B] = 1
            _upload(g.valid, vl)
            pos = torch.zeros(g.bp, dtype=torch.int32)
            pos[:B] = torch.tensor(lens, dtype=torch.int32)
            _upload(g.positions, pos)
            _upload(g.context_lens, pos + vl)
            self.set_order(g, lens)
            if grouped and g.groups_fit:
                self.set_groups(g, tables, [n + params.max_new_tokens for n in lens], nshared)
                if _DECODE_DUMP:
                    self._dump_decode(g, tables, lens, nshared, params)
            if not greedy:
                g.inv_temp.fill_(1.0 / params.temperature)
                g.top_k.fill_(params.top_k)
                g.top_p.fill_(params.top_p)
                if params.seed:
                    torch.manual_seed(params.seed)
            first = logits if greedy else self._select(logits, g)
            gen = torch.empty(B, params.max_new_tokens, dtype=torch.long, device=dev)
            gen[:, 0] = first
            tok = torch.zeros(g.bp, dtype=torch.int32, device=dev)
            tok[:B] = first.int()
            g.tokens.copy_(tok)
            if cuda:
                ev[1].record()
            t1 = time.perf_counter()
            if self.use_graphs and g.graph is None and params.max_new_tokens > 1:
                if cuda:  # this stream only: a pipelined prep stream keeps running
                    torch.cuda.current_stream().synchronize()
                self._capture(g)
            sp_dec = tracing.span("engine.decode_enqueue", steps=params.max_new_tokens - 1)
            sp_dec.__enter__()
            for step in range(1, params.max_new_tokens):
                if on_step is not None:
                    on_step(step, params.max_new_tokens)
                if g.graph is not None:
                    g.graph.replay()
                else:
                    self._step_body(g)
                gen[:, step] = g.out[:B]
            sp_dec.__exit__(None, None, None)
            if cuda:
                host = torch.empty(gen.shape, dtype=gen.dtype, pin_memory=True)
                host.copy_(gen, non_blocking=True)
            else:
                host = gen
            ar_err = comm.collective_error_snapshot()
            if cuda:
                ev[2].record()
        except BaseException:
            self.release(r)
            raise
        self.stats.prompt_tokens += sum(lens)
        self.stats.generated_tokens += B * params.max_new_tokens
        return Launched(r, host, ev, params, t0, t1, ar_err)

    def _dump_decode(self, g: _DecodeGraph, tables, lens, nshared: int, params: SamplingParams) -> None:
        """Diagnostics: the decode attention inputs of one cascade batch, for replaying the
        grouped kernel on its real block layout outside the engine."""
        if _DECODE_DUMP_SKIP[0] > 0:
            _DECODE_DUMP_SKIP[0] -= 1
            return
        _DECODE_DUMP_SKIP[0] = 1 << 30
        os.makedirs(_DECODE_DUMP, exist_ok=True)
        torch.save({"tables": tables, "lens": lens, "nshared": nshared, "bp": g.bp,
                    "groups": g.groups.cpu(), "max_new_tokens": params.max_new_tokens,
                    "block_size": self.block_size, "num_blocks": self.kv.caches[0][0].shape[0],
                    "max_blocks_per_seq": self.max_blocks_per_seq, "hq": self.model.hq, "hkv": self.model.hkv,
                    "head_dim": self.cfg.head_dim, "cascade_chunks": self._cascade_chunks(g.bp),
                    "inline": _inline_prefix_on() and not _defer_groups_on()},
                   os.path.join(_DECODE_DUMP, "decode_batch.pt"))

    def collect(self, h: "Launched") -> list[list[int]]:
        """Wait for a :meth:`launch`ed batch, free its KV blocks and return its tokens."""
        with tracing.span("engine.collect", seqs=h.reservation.n):
            return self._collect(h)

    def _collect(self, h: "Launched") -> list[list[int]]:
        try:
            if h.events is not None:
                h.events[2].synchronize()
                self.stats.prefill_s += h.events[0].elapsed_time(h.events[1]) / 1e3
                self.stats.decode_s += h.events[1].elapsed_time(h.events[2]) / 1e3
            else:
                t2 = time.perf_counter()
                self.stats.prefill_s += h.t1 - h.t0
                self.stats.decode_s += t2 - h.t1
            # a TP peer that never arrived leaves garbage tokens: fail, never return them
            comm.raise_on_collective_error(h.ar_err)
            result = h.host.tolist()
        finally:
            self.release(h.reservation)
        if h.params.stop_on_eos:
            eos = self.cfg.eos_token_id
            result = [r[: r.index(eos) + 1] if eos in r else r for r in result]
        return result
