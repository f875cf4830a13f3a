"""Worker for test_custom_ar_gpu: one rank of a 2-rank group (both on cuda:0 on the
1-GPU box; gloo only exchanges the IPC handles).  Exits non-zero on a mismatch."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("AR_DEVICE", "0")))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from docqa_amd.parallel.custom_ar import CustomAllReduce

    car = CustomAllReduce(max_bytes=4 << 20)
    for it in range(12):
        for n in (8, 4096, 64 * 4096, 2 << 20):
            xs = [torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + 10 * r + n % 7)).bfloat16()
                  for r in range(world)]
            ref = sum(x.float() for x in xs)
            out = car.all_reduce(xs[rank].cuda()).float().cpu()
            err = (out - ref).abs().max().item()
            tol = 0.02 * ref.abs().max().item() + 0.02
            if err > tol:
                print(f"rank {rank} it {it} n {n}: max err {err} > {tol}", flush=True)
                sys.exit(3)
    # HIP-graph replay advances the device-side epochs
    x = torch.full((4096,), float(rank + 1), device="cuda", dtype=torch.bfloat16)
    car.all_reduce(x)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            y = car.all_reduce(x)
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    expect = world * (world + 1) / 2
    if not torch.all(y.float() == expect):
        print(f"rank {rank}: graph replay gave {y[:4].tolist()} != {expect}", flush=True)
        sys.exit(4)
    car.check()
    dist.barrier()
    car.close()
    dist.destroy_process_group()
    print(f"rank {rank} ok", flush=True)


if __name__ == "__main__":
    main()
