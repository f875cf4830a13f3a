"""Tensor-parallel all-reduce over IPC-mapped peer memory (csrc/kernels/allreduce.hip) with
the residual add + RMSNorm that follows every row-parallel projection fused in.

Every rank reads its peers' staging buffers directly, so all 7 xGMI links of an MI355X
carry data at once instead of a ring's one link per step:
  * one-shot (messages <= ``oneshot_max_bytes``, latency-bound decode all-reduces): each
    rank sums all N staging buffers itself -- one cross-rank barrier;
  * two-shot (larger messages: decode at big batch, prefill): reduce-scatter of column
    chunks + all-gather -- 2 (N-1)/N of the message over xGMI instead of N-1.
The split-K fp32 slabs of the decode GEMMs go in directly (summed in registers on the
way into the staging buffer), so a row-parallel projection costs one GEMM launch and one
all-reduce launch that already writes the next layer's normed input.

Setup (once per TP group): each rank allocates an uncached staging + flag region, exports
its HIP IPC handle, the handles are exchanged with ``all_gather_object`` over the group,
and every rank maps its peers' regions; a self-test all-reduce then checks the mapping
before the caller relies on it (parallel/comm.py falls back to RCCL otherwise).  Calls are
HIP-graph capturable: the call epoch lives in device memory.

Reference parity: none (the reference has no collectives); this is the
custom all-reduce of SURVEY.md §2.3 / §5.8.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

ONESHOT, TWOSHOT, GATHER = 0, 1, 2


class CollectiveError(RuntimeError):
    """A TP collective did not complete (a peer was late past the bound or dead): every
    output of the step is garbage.  The serving loop treats it as fatal for the process
    (parallel/health.py, EXIT_COLLECTIVE_HANG) -- the launcher re-forms the group."""


def _agree(ok: bool, group, device) -> bool:
    """True only if ``ok`` on every rank of ``group`` (MIN all-reduce: a collective decision)."""
    on_gpu = dist.get_backend(group) != "gloo"
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device if on_gpu else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    return bool(flag.item())


class CustomAllReduce:
    def __init__(self, group=None, max_bytes: int = 64 << 20, device=None,
                 oneshot_max_bytes: int | None = None, timeout_ms: float | None = None):
        from .. import ops

        ops.load_native()
        self.nat = torch.ops.docqa
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > 8:
            raise ValueError("the IPC all-reduce supports up to 8 ranks (one xGMI hive)")
        self.device = torch.device(device or f"cuda:{torch.cuda.current_device()}")
        self.max_elems = max_bytes // 2 // 8 * 8
        if oneshot_max_bytes is None:
            oneshot_max_bytes = int(os.environ.get("DOCQA_AR_ONESHOT_MAX", str(256 << 10)))
        self.oneshot_max_bytes = oneshot_max_bytes
        # how long a workgroup waits for a late peer before it records which one and gives up
        # (the step then fails loudly: check() / raise_if()).  One process per GPU arrives
        # within microseconds; several processes on ONE GPU (tests, --share-gpu) must run
        # with GPU_MAX_HW_QUEUES=1 or a rank's queue may stay unmapped while the others spin
        # (allreduce.hip header; profiles/r4_ar_skew_*)
        # ``timeout_ms`` overrides it per instance: the data-parallel shard gathers
        # (index/sharded.py) meet ranks that are NOT in lockstep and wait much longer
        if timeout_ms is None:
            timeout_ms = float(os.environ.get("DOCQA_AR_TIMEOUT_MS", "500"))
        self.timeout_us = int(float(timeout_ms) * 1000)
        # every rank runs the same collective sequence whatever fails locally, so a failure
        # on one rank becomes the same decision on all of them (no rank left in a barrier)
        self.own, self.regions, self._opened = 0, [], []
        err: Exception | None = None
        handle = None
        try:
            self.own = self.nat.ar_alloc(self.nat.ar_region_bytes(self.max_elems))
            handle = self.nat.ar_ipc_handle(self.own).tolist()
        except Exception as e:  # noqa: BLE001 - reported collectively below
            err = e
        handles = [None] * self.world
        dist.all_gather_object(handles, handle, group=group)
        if err is None:
            try:
                if any(h is None for h in handles):
                    raise RuntimeError("a peer could not export its IPC handle")
                for r, h in enumerate(handles):
                    if r == self.rank:
                        self.regions.append(self.own)
                    else:
                        p = self.nat.ar_ipc_open(torch.tensor(h, dtype=torch.uint8))
                        self._opened.append(p)
                        self.regions.append(p)
            except Exception as e:  # noqa: BLE001
                err = e
        self.ctr = torch.zeros(4, dtype=torch.int32, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        if not _agree(err is None, group, self.device):
            self.close()
            raise RuntimeError(f"custom all-reduce setup failed on {'this rank' if err else 'a peer'}: {err}")

    # ------------------------------------------------------------------ capability
    def _fits(self, M: int, H: int, mode: int) -> bool:
        return M * H <= self.max_elems and H % 8 == 0 and (mode == ONESHOT or H % (8 * self.world) == 0)

    def mode_for(self, M: int, H: int) -> int:
        return ONESHOT if M * H * 2 <= self.oneshot_max_bytes or H % (8 * self.world) else TWOSHOT

    def supports(self, t: torch.Tensor) -> bool:
        if not (t.is_cuda and t.is_contiguous() and t.dim() >= 1):
            return False
        H = t.shape[-1]
        if t.dtype == torch.bfloat16:
            M = t.numel() // H
        elif t.dtype == torch.float32 and t.dim() == 3:   # split-K slabs [S, M, H]
            M = t.shape[1]
        else:
            return False
        return self._fits(M, H, self.mode_for(M, H))

    # ------------------------------------------------------------------ collectives
    def all_reduce(self, t: torch.Tensor, mode: int | None = None) -> torch.Tensor:
        """Sum of ``t`` (bf16 [.., H] or fp32 slabs [S, M, H]) over the group: a new bf16
        tensor; ``t`` is not modified."""
        slabs = t.dtype == torch.float32
        H = t.shape[-1]
        M = t.shape[1] if slabs else t.numel() // H
        mode = self.mode_for(M, H) if mode is None else mode
        return self.nat.ar_run(t, slabs, None, None, 0.0, self.rank, self.regions, self.max_elems, mode,
                               self.ctr, self.err, self.timeout_us)

    def reduce_add_rmsnorm(self, t: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                           mode: int | None = None) -> torch.Tensor:
        """residual <- residual + allreduce(t) (in place, bf16); returns rmsnorm(residual) * w
        -- ops.add_rmsnorm over the group's summed partials in one launch."""
        slabs = t.dtype == torch.float32
        H = t.shape[-1]
        M = t.shape[1] if slabs else t.numel() // H
        mode = self.mode_for(M, H) if mode is None else mode
        return self.nat.ar_run(t, slabs, residual, w, float(eps), self.rank, self.regions, self.max_elems,
                               mode, self.ctr, self.err, self.timeout_us)

    def all_gather_raw(self, t: torch.Tensor) -> torch.Tensor:
        """All-gather of any contiguous GPU tensor whose byte size is a multiple of 16:
        [world, *t.shape], bit-exact (the payload travels as raw 16-bit words) -- the
        vocab-parallel LM head's (value, id) candidates inside a captured decode graph."""
        nb = t.numel() * t.element_size()
        if nb % 16 or nb // 2 > self.max_elems:
            raise ValueError("all_gather_raw: payload must be a multiple of 16 bytes and fit the staging area")
        words = t.contiguous().view(torch.bfloat16).view(1, nb // 2)
        out = self.nat.ar_run(words, False, None, None, 0.0, self.rank, self.regions, self.max_elems, GATHER,
                              self.ctr, self.err, self.timeout_us)
        return out.view(t.dtype).view(self.world, *t.shape)

    def self_test(self) -> bool:
        """Both modes on a small tensor against the exact sum; False on any mismatch or a
        peer that never arrived (every rank runs it collectively)."""
        ok = True
        for mode in (ONESHOT, TWOSHOT):
            H = 8 * self.world * 4
            x = torch.full((3, H), float(self.rank + 1), device=self.device, dtype=torch.bfloat16)
            y = self.all_reduce(x, mode)
            torch.cuda.synchronize(self.device)
            ok = ok and bool(torch.all(y.float() == self.world * (self.world + 1) / 2))
        ids = torch.arange(4, device=self.device, dtype=torch.int64) + 1000 * self.rank
        gat = self.all_gather_raw(ids)
        ok = ok and bool(torch.equal(gat.cpu(), torch.arange(4).repeat(self.world, 1)
                                     + 1000 * torch.arange(self.world)[:, None]))
        ok = ok and int(self.err.item()) == 0
        return _agree(ok, self.group, self.device)

    # ------------------------------------------------------------------ failure surfacing
    def snapshot(self) -> torch.Tensor:
        """Stream-ordered, non-blocking copy of the error word into pinned host memory:
        taken behind a step's kernels and read (``raise_if``) after the step's existing host
        sync, so surfacing a late or dead peer costs no extra synchronisation."""
        h = torch.empty(1, dtype=torch.int32, pin_memory=True)
        h.copy_(self.err, non_blocking=True)
        return h

    @staticmethod
    def describe(word: int) -> str:
        word &= 0xFFFFFFFF
        return (f"custom all-reduce: rank {(word >> 1) & 7} never arrived (phase {(word >> 4) & 1}, "
                f"call epoch {word >> 8}); the step's results are invalid")

    def raise_if(self, snap: torch.Tensor | None) -> None:
        if snap is not None and int(snap[0]):
            raise CollectiveError(self.describe(int(snap[0])))

    def check(self) -> None:
        """Synchronous form (tests, between requests)."""
        w = int(self.err.item())
        if w:
            raise CollectiveError(self.describe(w))

    def max_wait_us(self) -> int:
        """Longest time any workgroup waited for a peer since the counters were zeroed."""
        return int(self.ctr[2].item())

    def close(self) -> None:
        for p in getattr(self, "_opened", []):
            self.nat.ar_ipc_close(p)
        self._opened = []
        if self.own:
            torch.cuda.synchronize(self.device)
            self.nat.ar_free(self.own)
            self.own = 0
