"""Which host->device upload forms block the host while the GPU stream is still busy?
(Decides how the engine stages its per-batch uploads behind a queued decode.)
Usage: python scripts/h2d_block_probe.py"""
import json
import time

import torch

dev = "cuda"
a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)


def busy(ms=60):
    """queue ~ms of GPU work on the current stream"""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        a @ a
    torch.cuda.synchronize()
    per = (time.perf_counter() - t0) / 200
    n = max(1, int(ms / 1e3 / per))
    for _ in range(n):
        a @ a
    return n * per * 1e3


def host_ms(fn, reps=8):
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) * 1e3 / reps


src = list(range(4096))
cpu = torch.tensor(src, dtype=torch.int32)
dst = torch.empty(4096, dtype=torch.int32, device=dev)
pinned = torch.empty(4096, dtype=torch.int32, pin_memory=True)
res = {}
forms = {
    "torch.tensor(list, device=cuda)": lambda: torch.tensor(src, dtype=torch.int32, device=dev),
    "pageable .to(cuda, non_blocking)": lambda: cpu.to(dev, non_blocking=True),
    "pageable copy_ non_blocking": lambda: dst.copy_(cpu, non_blocking=True),
    "fresh pin_memory() + copy_": lambda: dst.copy_(cpu.clone().pin_memory(), non_blocking=True),
    "persistent pinned + copy_": lambda: dst.copy_(pinned, non_blocking=True),
    "torch.empty(pin_memory=True)": lambda: torch.empty(65536, dtype=torch.int32, pin_memory=True),
}
for name, fn in forms.items():
    q = busy()
    res[name] = {"gpu_queued_ms": round(q, 1), "host_ms_per_call": round(host_ms(fn), 3)}
    torch.cuda.synchronize()
    print(json.dumps({name: res[name]}), flush=True)
