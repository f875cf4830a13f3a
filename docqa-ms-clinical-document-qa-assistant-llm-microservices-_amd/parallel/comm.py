"""Process-group plumbing: one process per GPU, torch.distributed over RCCL ("nccl"
backend on ROCm = RCCL over xGMI) on the GPU box, gloo on CPU for CI.

Topology on one MI355X node: 8 GPUs fully connected by xGMI (7 point-to-point links
per GPU).  We split WORLD into

  * tensor-parallel groups (contiguous ranks, TP in {1, 2, 4, 8}) for the generator's
    per-layer all-reduces, and
  * data-parallel groups (ranks with equal TP index) for request-level replicas and
    the sharded vector index (all-gather of per-shard top-k).

Reference parity: the reference has no collectives at all; scale-out
there is competing AMQP consumers (deid-service/anonymizer.py:97).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class ParallelState:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    tp_size: int = 1
    tp_rank: int = 0
    dp_size: int = 1
    dp_rank: int = 0
    tp_group: object = None
    dp_group: object = None
    backend: str = "none"
    # CPU (gloo) group over the same ranks as tp_group: host-side control messages
    # (the lockstep serving loop's broadcasts) that must not touch the GPU stream
    tp_cpu_group: object = None

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1


_STATE = ParallelState()


def state() -> ParallelState:
    return _STATE


def init_distributed(tp_size: int = 1, backend: str | None = None, timeout_s: int = 600,
                     store=None) -> ParallelState:
    """Initialise torch.distributed from torchrun env vars (RANK/WORLD_SIZE/MASTER_*).

    Safe to call without a launcher: falls back to a single-process state.  ``store``: an
    existing rendezvous store (parallel/health.py:reinit re-forms the groups on it).
    """
    global _STATE
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and not dist.is_initialized():
        _STATE = ParallelState(tp_size=1, backend="none")
        return _STATE
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if os.environ["MASTER_ADDR"] in ("127.0.0.1", "localhost") and os.path.exists("/sys/class/net/lo"):
        # single node: gloo (the process group of CPU / shared-GPU runs and the side groups
        # of RCCL runs) otherwise binds the interface the hostname resolves to, which in a
        # container may be unreachable -- a rank then joins the mesh with 0 peers
        os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
    if not dist.is_initialized():
        kw = {}
        if store is not None:
            kw["store"] = store
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local_rank)
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    if world % tp_size != 0:
        raise ValueError(f"world size {world} not divisible by tp {tp_size}")
    dp_size = world // tp_size
    tp_group = dp_group = tp_cpu = None
    # every rank must create every group in the same order
    for d in range(dp_size):
        ranks = list(range(d * tp_size, (d + 1) * tp_size))
        g = dist.new_group(ranks) if tp_size > 1 else None
        gc = (dist.new_group(ranks, backend="gloo") if backend != "gloo" else g) if tp_size > 1 else None
        if rank in ranks:
            tp_group, tp_cpu = g, gc
    for t in range(tp_size):
        ranks = list(range(t, world, tp_size))
        g = dist.new_group(ranks) if dp_size > 1 else None
        if rank in ranks:
            dp_group = g
    _STATE = ParallelState(rank=rank, world_size=world, local_rank=local_rank, tp_size=tp_size,
                           tp_rank=rank % tp_size, dp_size=dp_size, dp_rank=rank // tp_size,
                           tp_group=tp_group, dp_group=dp_group, backend=backend, tp_cpu_group=tp_cpu)
    if tp_size > 1 and backend == "nccl" and os.environ.get("DOCQA_CUSTOM_AR", "1") == "1":
        # every TP group sets up its IPC all-reduce at once (collective within the group)
        enable_custom_all_reduce()
    return _STATE


def set_state(s: ParallelState) -> None:
    global _STATE
    _STATE = s


_CUSTOM_AR = None


def enable_custom_all_reduce(max_bytes: int | None = None, force: bool = False):
    """Route the TP all-reduces through the IPC all-reduce (parallel/custom_ar.py: one-shot /
    two-shot over all xGMI links, residual + RMSNorm fused) for every message that fits
    ``max_bytes`` (default 128 MB = 8192 prefill tokens of a 8192-wide model; env
    DOCQA_AR_MAX_MB); RCCL keeps everything else.  Called
    by ``init_distributed`` at TP > 1 on RCCL unless DOCQA_CUSTOM_AR=0; a failed IPC mapping
    or self-test leaves RCCL in charge (returns None)."""
    global _CUSTOM_AR
    s = _STATE
    if s.tp_size > 1 and (s.backend == "nccl" or force) and _CUSTOM_AR is None:
        from .custom_ar import CustomAllReduce
        if max_bytes is None:
            max_bytes = int(os.environ.get("DOCQA_AR_MAX_MB", "128")) << 20
        car = None
        try:
            car = CustomAllReduce(group=s.tp_group, max_bytes=max_bytes)
            ok = car.self_test()
        except Exception as e:  # pragma: no cover - depends on the node's IPC support
            print(f"[comm] custom all-reduce unavailable ({e}); using RCCL", flush=True)
            ok = False
        if ok:
            _CUSTOM_AR = car
        elif car is not None:
            car.close()
    return _CUSTOM_AR


def custom_all_reduce():
    return _CUSTOM_AR


def collective_error_snapshot():
    """Non-blocking, stream-ordered copy of the IPC all-reduce's error word (None when the
    custom all-reduce is not in use).  Take it right after a step's kernels are enqueued and
    pass it to :func:`raise_on_collective_error` after the step's own host sync."""
    return _CUSTOM_AR.snapshot() if _CUSTOM_AR is not None else None


def raise_on_collective_error(snap) -> None:
    """Raise ``CollectiveError`` when the snapshot says a peer never arrived: the step's
    outputs are garbage, and the caller must not hand them out."""
    if snap is not None and _CUSTOM_AR is not None:
        _CUSTOM_AR.raise_if(snap)


def tp_all_reduce(t: torch.Tensor) -> torch.Tensor:
    s = _STATE
    if s.tp_size > 1:
        if _CUSTOM_AR is not None and _CUSTOM_AR.supports(t):
            return _CUSTOM_AR.all_reduce(t)
        dist.all_reduce(t, group=s.tp_group)
    return t


def tp_add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    """The end of a row-parallel projection: residual <- residual + sum over the TP group of
    ``x`` (a bf16 partial [M, H] or the GEMM's fp32 split-K slabs [S, M, H]), returns
    rmsnorm(residual) * w.  TP = 1: the fused split-K consumer / add_rmsnorm kernel; TP > 1:
    one launch of the IPC all-reduce with the add + norm in its epilogue, else RCCL
    all-reduce + add_rmsnorm."""
    from .. import ops

    slabs = x.dim() == residual.dim() + 1     # split-K slabs [S, M, H] vs a partial [M, H]
    s = _STATE
    if s.tp_size == 1:
        return ops.add_rmsnorm_splitk(x, residual, w, eps) if slabs else ops.add_rmsnorm(x, residual, w, eps)
    if _CUSTOM_AR is not None and _CUSTOM_AR.supports(x):
        return _CUSTOM_AR.reduce_add_rmsnorm(x, residual, w, eps)
    # fp32 slabs are summed across the group in fp32 and rounded once, as the TP = 1 GEMM
    # rounds its fp32 accumulator once (rounding each rank's partial first flips bf16 ties)
    y = x.float().sum(0) if slabs else x.contiguous()
    dist.all_reduce(y, group=s.tp_group)
    return ops.add_rmsnorm(y.to(residual.dtype), residual, w, eps)


def tp_argmax(vals: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
    """Greedy pick over a vocab-parallel LM head: each rank's row-best (value, global id) ->
    the group's best id, ties to the lowest id (torch.argmax order) -- one int64 MAX
    all-reduce of packed keys [order-preserving value bits | ~id] instead of gathering
    [B, vocab] logits or (value, id) pairs."""
    s = _STATE
    v = vals.float().contiguous().view(torch.int32).to(torch.int64)
    ordered = torch.where(v >= 0, v, v ^ 0x7FFFFFFF)          # int32 range, monotonic in the float
    key = ordered * (1 << 32) + ((1 << 32) - 1 - ids.to(torch.int64))   # exact in int64
    if s.tp_size > 1:
        if _CUSTOM_AR is not None and key.is_cuda and key.numel() % 2 == 0:
            # IPC all-gather of the [R] keys + a local max: graph-capturable on any backend
            key = _CUSTOM_AR.all_gather_raw(key).max(dim=0).values
        elif _CUSTOM_AR is not None and key.is_cuda:
            pad = torch.cat([key, key[:1]])
            key = _CUSTOM_AR.all_gather_raw(pad).max(dim=0).values[: key.numel()]
        else:
            dist.all_reduce(key, op=dist.ReduceOp.MAX, group=s.tp_group)
    return (1 << 32) - 1 - torch.remainder(key, 1 << 32)


def tp_all_gather_last(t: torch.Tensor) -> torch.Tensor:
    """All-gather along the last dim across the TP group (vocab-parallel logits)."""
    s = _STATE
    if s.tp_size == 1:
        return t
    parts = [torch.empty_like(t) for _ in range(s.tp_size)]
    dist.all_gather(parts, t.contiguous(), group=s.tp_group)
    return torch.cat(parts, dim=-1)


def dp_all_gather(t: torch.Tensor) -> list[torch.Tensor]:
    s = _STATE
    if s.dp_size == 1:
        return [t]
    parts = [torch.empty_like(t) for _ in range(s.dp_size)]
    dist.all_gather(parts, t.contiguous(), group=s.dp_group)
    return parts


def barrier() -> None:
    if dist.is_initialized():
        if _STATE.backend == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def destroy() -> None:
    global _STATE, _CUSTOM_AR
    if _CUSTOM_AR is not None:
        _CUSTOM_AR.close()
        _CUSTOM_AR = None
    if dist.is_initialized():
        dist.destroy_process_group()
    _STATE = ParallelState()
