"""Worker for test_custom_ar_gpu: one rank of an N-rank group (all on cuda:0 on the 1-GPU
box, reaching each other's staging through HIP IPC; gloo only exchanges the handles).
Checks the IPC all-reduce (csrc/kernels/allreduce.hip) in both modes, bf16 partials and
fp32 split-K slabs, plain and with the fused residual add + RMSNorm, against the fp32
PyTorch reference of the same op; then HIP-graph replays.  Exits non-zero on a mismatch."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import torch.distributed as dist


def _inputs(it, M, H, S, world, slabs):
    """Every rank's partial (the same on every rank: each builds all of them)."""
    parts = []
    for r in range(world):
        g = torch.Generator().manual_seed(1000 * it + 10 * r + M + H + S)
        if slabs:
            parts.append(torch.randn(S, M, H, generator=g))
        else:
            parts.append(torch.randn(M, H, generator=g).bfloat16())
    return parts


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(int(os.environ.get("AR_DEVICE", "0")))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from docqa_amd.ops import reference as ref
    from docqa_amd.parallel.custom_ar import ONESHOT, TWOSHOT, CustomAllReduce

    car = CustomAllReduce(max_bytes=8 << 20)
    assert car.self_test(), "self test failed"
    it = 0
    for mode in (ONESHOT, TWOSHOT):
        for (M, H) in ((1, 256), (3, 1024), (64, 1024), (300, 512), (1024, 2048)):
            for slabs, S in ((False, 0), (True, 1), (True, 3)):
                for fused in (False, True):
                    it += 1
                    parts = _inputs(it, M, H, S, world, slabs)
                    # each rank's slabs summed in slab order (the kernel's order), rounded to bf16
                    # (its staging), then the ranks summed in rank order in fp32
                    def own(p):
                        if not slabs:
                            return p.float()
                        acc = p[0].clone()
                        for sl in range(1, p.shape[0]):
                            acc = acc + p[sl]
                        return acc
                    total = sum(own(p).bfloat16().float() for p in parts)
                    g = torch.Generator().manual_seed(it)
                    res0 = torch.randn(M, H, generator=g).bfloat16()
                    w = (1 + 0.1 * torch.randn(H, generator=g)).bfloat16()
                    x = parts[rank].cuda()
                    if fused:
                        res = res0.cuda()
                        out = car.reduce_add_rmsnorm(x, res, w.cuda(), 1e-5, mode=mode)
                        rres = res0.clone()
                        expect = ref.add_rmsnorm(total.bfloat16(), rres, w, 1e-5).float()
                        # every mode rounds the cross-rank sum to bf16 before the residual
                        # add, so the updated residual is bf16(bf16(sum) + r) bit for bit -- one-shot,
                        # two-shot and RCCL + add_rmsnorm alike
                        if not torch.equal(res.cpu(), rres):
                            err_r = (res.float().cpu() - rres.float()).abs().max().item()
                            print(f"rank {rank} mode {mode} M {M} H {H} S {S}: residual not bit-exact "
                                  f"(max err {err_r})", flush=True)
                            sys.exit(3)
                    else:
                        out = car.all_reduce(x, mode=mode)
                        expect = total
                    got = out.float().cpu().view_as(expect)
                    err = (got - expect).abs().max().item()
                    tol = 0.02 * expect.abs().max().item() + 0.02
                    if err > tol:
                        print(f"rank {rank} mode {mode} M {M} H {H} S {S} fused {fused}: err {err} > {tol}",
                              flush=True)
                        sys.exit(3)
    # HIP-graph replay advances the device-side call epoch
    for mode in (ONESHOT, TWOSHOT):
        x = torch.full((64, 1024), float(rank + 1), device="cuda", dtype=torch.bfloat16)
        car.all_reduce(x, mode=mode)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            with torch.cuda.graph(gr, stream=s):
                y = car.all_reduce(x, mode=mode)
        for _ in range(7):
            gr.replay()
        torch.cuda.synchronize()
        expect = world * (world + 1) / 2
        if not torch.all(y.float() == expect):
            print(f"rank {rank}: graph replay mode {mode} gave {y.flatten()[:4].tolist()} != {expect}", flush=True)
            sys.exit(4)
    car.check()
    dist.barrier()
    car.close()
    dist.destroy_process_group()
    print(f"rank {rank} ok", flush=True)


if __name__ == "__main__":
    main()
