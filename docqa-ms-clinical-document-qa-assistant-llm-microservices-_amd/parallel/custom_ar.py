"""One-shot all-reduce over IPC-mapped peer memory (csrc/kernels/allreduce.hip) for the
tensor-parallel decode all-reduces: every rank reads all peers' staging buffers at once
over xGMI's point-to-point links instead of a ring's 2(N-1) dependent hops.

Setup (once per TP group): each rank allocates an uncached staging+flag region, exports
its HIP IPC handle, the handles are exchanged with ``all_gather_object`` over the group,
and every rank maps its peers' regions.  ``all_reduce(x)`` is then one kernel launch
(HIP-graph capturable: the barrier epochs live in device memory).  Payloads above
``max_bytes``, non-bf16 tensors and CPU tensors go to RCCL (torch.distributed).

Reference parity: none (the reference has no collectives); this is the
custom all-reduce of SURVEY.md §2.3 / §5.8.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

_MAX_WG = 128


class CustomAllReduce:
    def __init__(self, group=None, max_bytes: int = 8 << 20, device=None):
        from .. import ops

        ops.load_native()
        self.nat = torch.ops.docqa
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > 8:
            raise ValueError("one-shot all-reduce supports up to 8 ranks (one xGMI hive)")
        self.device = torch.device(device or f"cuda:{torch.cuda.current_device()}")
        self.max_elems = max_bytes // 2 // 8 * 8
        nbytes = self.nat.ar_region_bytes(self.max_elems)
        self.own = self.nat.ar_alloc(nbytes)
        handle = self.nat.ar_ipc_handle(self.own)
        handles = [None] * self.world
        dist.all_gather_object(handles, handle.tolist(), group=group)
        self.regions = []
        self._opened = []
        for r, h in enumerate(handles):
            if r == self.rank:
                self.regions.append(self.own)
            else:
                p = self.nat.ar_ipc_open(torch.tensor(h, dtype=torch.uint8))
                self._opened.append(p)
                self.regions.append(p)
        self.epochs = torch.zeros(_MAX_WG, dtype=torch.int32, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        dist.barrier(group=group)

    def supports(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous()
                and t.numel() % 8 == 0 and t.numel() <= self.max_elems)

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        """Sum of ``t`` over the group (a new tensor; ``t`` is not modified)."""
        return self.nat.ar_oneshot(t, self.rank, self.regions, self.max_elems, self.epochs, self.err)

    def check(self) -> None:
        if int(self.err.item()):
            raise RuntimeError("custom all-reduce: a peer never arrived (spin limit hit)")

    def close(self) -> None:
        for p in self._opened:
            self.nat.ar_ipc_close(p)
        self._opened = []
        if self.own:
            torch.cuda.synchronize(self.device)
            self.nat.ar_free(self.own)
            self.own = 0
