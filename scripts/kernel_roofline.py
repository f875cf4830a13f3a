"""Per-kernel roofline table of the headline decode step from a rocprofv3 --stats run.

Reads ``run_kernel_stats.csv`` (average us per call) and the bench JSON line (for the KV
bytes the grouped attention reads per layer) and prints a markdown table: us per call,
calls per decode step, bytes and FLOPs per call (model-derived for Llama-3-8B at batch 256,
bf16 weights, bf16 split-K slabs (DOCQA_SLAB_BF16 default; fp32 when the stats show the
fp32-slab kernels), the splits ops.mid_plan picks), TB/s and TFLOP/s.  Bytes
count each operand once (HBM-level traffic): L2 re-reads of the activations are not counted.

Usage: python scripts/kernel_roofline.py <run_kernel_stats.csv> <bench.log with the JSON line>
"""
import csv
import json
import sys

MB = 1e6
B, H, I, V = 256, 4096, 14336, 128256
QKV = 6144


def rows(kv_mb, sb=2):
    """sb: split-K slab element bytes (2: bf16 slabs, mgemm EPI 4; 4: fp32, EPI 1)."""
    w = lambda n, k: n * k * 2            # bf16 weight bytes
    x = lambda k: B * k * 2               # bf16 activation bytes
    slab = lambda s, n: s * B * n * sb    # split-K slabs
    epi = 4 if sb == 2 else 1
    pt = ", unsigned short" if sb == 2 else ", float"
    qkv = (w(QKV, H) + x(H) + slab(4, QKV), 2 * B * H * QKV)
    down = (w(H, I) + x(I) + slab(8, H), 2 * B * I * H)
    return [
        # (label, name pattern, calls per step, bytes, flops)
        ("gate|up + SwiGLU (mgemm cfg 2, S=1)", "mgemm_kernel<2, 128", 32,
         w(2 * I, H) + x(H) + x(I), 2 * B * H * 2 * I),
        ("QKV (S=4) / down (S=8) (mgemm cfg 2), mean of the two", f"mgemm_kernel<{epi}, 128", 64,
         (qkv[0] + down[0]) / 2, (qkv[1] + down[1]) / 2),
        ("O (mgemm cfg 7, S=4)", f"mgemm_kernel<{epi}, 64", 32, w(H, H) + x(H) + slab(4, H), 2 * B * H * H),
        ("LM head + argmax (mgemm cfg 6)", "mgemm_kernel<3, 256", 1, w(V, H) + x(H), 2 * B * H * V),
        ("grouped paged attention (wave kernel; distinct KV blocks once)", "paged_decode_group_wave_kernel", 32,
         kv_mb * MB, 0),
        ("down consumer: slabs + residual + RMSNorm", f"add_rmsnorm_splitk_kernel<2, 8{pt}", 32,
         slab(8, H) + 3 * x(H), 0),
        ("O consumer: slabs + residual + RMSNorm", f"add_rmsnorm_splitk_kernel<2, 4{pt}", 32,
         slab(4, H) + 3 * x(H), 0),
        ("QKV consumer: slabs + RoPE + KV write", f"rope_cache_kernel<true, 4{pt}", 32,
         slab(4, QKV) + x(H) + 2 * B * 1024 * 2, 0),
    ]


def main():
    stats = {r["Name"]: r for r in csv.DictReader(open(sys.argv[1]))}
    bench = next(json.loads(l) for l in open(sys.argv[2]) if l.startswith("{\"metric\""))
    kv_mb = float(bench.get("decode_attn_kv_mb_per_layer", 0.0))
    step_ms = bench["engine_ms_per_batch"]["decode"] / bench["config"]["max_new_tokens"]
    print(f"decode step {step_ms:.2f} ms (engine decode {bench['engine_ms_per_batch']['decode']:.1f} ms / "
          f"{bench['config']['max_new_tokens']} steps), grouped-attention KV {kv_mb:.1f} MB per layer\n")
    sb = 2 if any("mgemm_kernel<4," in n for n in stats) else 4
    print(f"split-K slabs: {'bf16' if sb == 2 else 'fp32'}\n")
    print("| kernel | us / call | calls / step | us / step | MB / call | TB/s | TFLOP/s |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    tot = 0.0
    for label, pat, calls, nbytes, flops in rows(kv_mb, sb):
        hit = [r for n, r in stats.items() if pat in n]
        if not hit:
            continue
        us = sum(float(r["TotalDurationNs"]) for r in hit) / sum(int(r["Calls"]) for r in hit) / 1e3
        tot += us * calls
        tf = f"{flops / us / 1e6:.0f}" if flops else "-"
        print(f"| {label} | {us:.1f} | {calls} | {us * calls:.0f} | {nbytes / MB:.1f} | "
              f"{nbytes / us / 1e6:.2f} | {tf} |")
    print(f"\nlisted kernels: {tot / 1e3:.2f} ms of the {step_ms:.2f} ms step")


if __name__ == "__main__":
    main()
