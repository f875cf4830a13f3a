"""Prefill attention probe: paged (prefix-cached) causal prefill at RAG shapes vs the
contiguous kernel, to locate the prefill-attention cost seen in the bench profile."""
import json
import math
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

from benchmarks.bench_kernels import timeit
from docqa_amd import ops


def main():
    assert ops.load_native()
    nat = torch.ops.docqa
    # PROBE_HEADS=64,8: the Llama-3-70B head layout (8 query heads per KV head)
    Hq, Hkv = (int(v) for v in os.environ.get("PROBE_HEADS", "32,8").split(","))
    D, BS = 128, 64
    scale = 1 / math.sqrt(D)
    for B, new, pre in [(128, 130, 448), (128, 130, 0), (64, 130, 448), (16, 600, 0), (128, 16, 448)]:
        W = (Hq + 2 * Hkv) * D
        T = B * new
        qkv = (torch.randn(T, W, device="cuda") * 0.5).bfloat16()
        cu = torch.arange(0, T + 1, new, device="cuda", dtype=torch.int32)
        flops = 4 * B * Hq * D * (new * pre + new * new / 2)
        if pre:
            maxb = (pre + new + BS - 1) // BS
            NB = B * maxb + 1
            kc = torch.randn(NB, Hkv, BS, D, device="cuda").bfloat16()
            vc = torch.randn_like(kc)
            bt = torch.arange(B * maxb, device="cuda", dtype=torch.int32).view(B, maxb)
            cs = torch.full((B,), pre, device="cuda", dtype=torch.int32)
            f = lambda: nat.flash_prefill_paged(qkv, cu, new, Hq, Hkv, D, scale, kc, vc, bt, cs)
        else:
            f = lambda: nat.flash_prefill(qkv, cu, new, Hq, Hkv, D, scale, True)
        t = timeit(f, iters=10)
        print(f"B={B} new={new} prefix={pre}: {t:.1f} us  {flops / t / 1e6:.1f} TFLOP/s", flush=True)
    # the bench's steady-state mix: new tokens 30..370 (mean ~90), cached prefix 320..768
    g = torch.Generator().manual_seed(0)
    B = 128
    news = (30 + torch.randint(0, 120, (B,), generator=g)).tolist()
    news[5] = 370
    pres = (64 * (5 + torch.randint(0, 8, (B,), generator=g))).tolist()
    W = (Hq + 2 * Hkv) * D
    T = sum(news)
    qkv = (torch.randn(T, W, device="cuda") * 0.5).bfloat16()
    cu = torch.tensor([0] + list(__import__("itertools").accumulate(news)), device="cuda", dtype=torch.int32)
    maxb = (max(p + n for p, n in zip(pres, news)) + BS - 1) // BS
    kc = torch.randn(B * maxb + 1, Hkv, BS, D, device="cuda").bfloat16()
    vc = torch.randn_like(kc)
    bt = torch.arange(B * maxb, device="cuda", dtype=torch.int32).view(B, maxb)
    cs = torch.tensor(pres, device="cuda", dtype=torch.int32)
    flops = sum(4 * Hq * D * (n * p + n * n / 2) for n, p in zip(news, pres))
    t = timeit(lambda: nat.flash_prefill_paged(qkv, cu, max(news), Hq, Hkv, D, scale, kc, vc, bt, cs), iters=10)
    print(f"bench-mix B={B} new mean={T / B:.0f} max={max(news)} prefix 320..768: {t:.1f} us  {flops / t / 1e6:.1f} TFLOP/s")


def replay(dump_dir: str):
    """Time the paged prefill kernel on the exact (cu_seqlens, cached lengths, block tables)
    the engine saved with DOCQA_PREFILL_DUMP=<dir>, with the real (shared) block ids and
    with the same lengths on private contiguous blocks."""
    import glob

    assert ops.load_native()
    nat = torch.ops.docqa
    Hq, Hkv, D, BS = 32, 8, 128, 64
    scale = 1 / math.sqrt(D)
    for f in sorted(glob.glob(f"{dump_dir}/prefill_*.pt")):
        d = torch.load(f, weights_only=True)
        cu, ctx, bt = d["cu"], d["ctx"], d["bt"]
        B = len(ctx)
        news = (cu[1:] - cu[:-1]).tolist()
        T = int(cu[-1])
        W = (Hq + 2 * Hkv) * D
        qkv = (torch.randn(T, W, device="cuda") * 0.5).bfloat16()
        nb = int(bt.max()) + 1
        maxb = bt.shape[1]
        kc = torch.randn(max(nb, B * maxb) + 1, Hkv, BS, D, device="cuda").bfloat16()
        vc = torch.randn_like(kc)
        flops = sum(4 * Hq * D * (n * p + n * n / 2) for n, p in zip(news, ctx.tolist()))
        cud, csd = cu.cuda(), ctx.cuda()
        uniq = len(set(bt[r, k].item() for r in range(B) for k in range((int(ctx[r]) + news[r] + BS - 1) // BS)))
        for name, table in (("real", bt.cuda()), ("private", torch.arange(B * maxb, dtype=torch.int32, device="cuda").view(B, maxb))):
            t = timeit(lambda: nat.flash_prefill_paged(qkv, cud, max(news), Hq, Hkv, D, scale, kc, vc, table, csd), iters=10)
            print(json.dumps({"file": f.split("/")[-1], "tables": name, "B": B, "new_sum": T, "new_max": max(news),
                              "ctx_mean": round(float(ctx.float().mean()), 1), "ctx_max": int(ctx.max()),
                              "unique_blocks": uniq, "us": round(t, 1), "tflops": round(flops / t / 1e6, 1)}), flush=True)


def replay_variants(dump_dir: str):
    """Which property of the real batch makes the paged prefill slow: subsets of the
    sequences, uniform new lengths, no cached prefix."""
    import glob

    assert ops.load_native()
    nat = torch.ops.docqa
    Hq, Hkv, D, BS = 32, 8, 128, 64
    scale = 1 / math.sqrt(D)
    f = sorted(glob.glob(f"{dump_dir}/prefill_*.pt"))[-1]
    d = torch.load(f, weights_only=True)
    news0, ctx0 = (d["cu"][1:] - d["cu"][:-1]).tolist(), d["ctx"].tolist()
    W = (Hq + 2 * Hkv) * D
    maxb = 40
    kc = torch.randn(128 * maxb + 1, Hkv, BS, D, device="cuda").bfloat16()
    vc = torch.randn_like(kc)

    def run(name, news, ctx):
        B = len(news)
        cu = torch.tensor([0] + list(__import__("itertools").accumulate(news)), dtype=torch.int32, device="cuda")
        T = int(cu[-1])
        qkv = (torch.randn(T, W, device="cuda") * 0.5).bfloat16()
        bt = torch.arange(B * maxb, dtype=torch.int32, device="cuda").view(B, maxb)
        cs = torch.tensor(ctx, dtype=torch.int32, device="cuda")
        flops = sum(4 * Hq * D * (n * p + n * n / 2) for n, p in zip(news, ctx))
        t = timeit(lambda: nat.flash_prefill_paged(qkv, cu, max(news), Hq, Hkv, D, scale, kc, vc, bt, cs), iters=10)
        print(json.dumps({"variant": name, "B": B, "new_sum": T, "new_max": max(news), "us": round(t, 1),
                          "tflops": round(flops / t / 1e6, 1)}), flush=True)

    run("real", news0, ctx0)
    for k in (16, 32, 64):
        run(f"first{k}", news0[:k], ctx0[:k])
    order = sorted(range(128), key=lambda i: -news0[i])
    run("longest16", [news0[i] for i in order[:16]], [ctx0[i] for i in order[:16]])
    run("shortest112", [news0[i] for i in order[16:]], [ctx0[i] for i in order[16:]])
    run("new_capped64", [min(n, 64) for n in news0], ctx0)
    run("ctx0", news0, [0] * 128)
    run("uniform", [sum(news0) // 128] * 128, [sum(ctx0) // 128 // 64 * 64] * 128)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--variants":
        replay_variants(sys.argv[2])
        sys.exit(0)
    if len(sys.argv) > 2 and sys.argv[1] == "--replay":
        replay(sys.argv[2])
    else:
        main()
