"""Can two RCCL ranks share one GPU on this pool?  torchrun --nproc-per-node 2 this file:
each rank binds cuda:0, runs an all_reduce and an all_gather over the nccl (RCCL) backend
and prints what it got.  Used to decide whether the one-GPU DP rehearsal of bench.py
(--share-gpu) can run on RCCL or must use gloo."""
import datetime
import os

import torch
import torch.distributed as dist

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60),
                        device_id=torch.device("cuda", 0))
x = torch.full((1024,), float(rank + 1), device="cuda")
dist.all_reduce(x)
parts = [torch.empty(4, device="cuda") for _ in range(world)]
dist.all_gather(parts, torch.full((4,), float(rank), device="cuda"))
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce {x[0].item()} (want {world * (world + 1) / 2}), "
      f"all_gather {[p[0].item() for p in parts]}", flush=True)
dist.destroy_process_group()
