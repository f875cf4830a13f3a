"""GPU occupancy of a serving run from a rocprofv3 kernel trace of the service process
(benchmarks/bench_serving.py --launch-prefix 'rocprofv3 --kernel-trace ...'): over the
middle of the loaded span (ends trimmed by --trim-s), the fraction of wall time with a
kernel running, the idle gaps by size and which kernels bracket the large ones, and the
kernel time split into prefill (pgemm / flash prefill / prefill norms) and decode.

Usage: python scripts/serve_trace.py <run_kernel_trace.csv> [--trim-s 2] [--min-gap-us 50]
"""
import argparse
import csv
from collections import Counter, defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--trim-s", type=float, default=2.0)
    ap.add_argument("--last-s", type=float, default=0.0,
                    help="analyse only the last this many seconds of the loaded span (the timed run; "
                         "the service's start-up graph captures and GEMM tuning come before it)")
    ap.add_argument("--min-gap-us", type=float, default=50.0)
    ap.add_argument("--skip-tuning", action="store_true", help="start after the last TunableOp flush")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # the loaded span: the longest run of kernels with no gap over 200 ms (service startup,
    # warm-up and shutdown are separated from it by idle seconds)
    spans, s0, last = [], rows[0][0], rows[0][1]
    for s, e, _ in rows[1:]:
        if s - last > 200e6:
            spans.append((s0, last))
            s0 = s
        last = max(last, e)
    spans.append((s0, last))
    lo, hi = max(spans, key=lambda x: x[1] - x[0])
    # the service's start-up (decode-graph captures, TunableOp tuning of their library GEMMs:
    # flush_icache between candidates) runs right before the load; start after its last kernel
    # per-second timeline of the span: all kernels, TunableOp candidate flushes, decode GEMMs
    per = defaultdict(lambda: [0, 0, 0])
    for s_, e_, n in rows:
        if lo <= s_ <= hi:
            b = per[int((s_ - lo) / 1e9)]
            b[0] += 1
            b[1] += "flush_icache" in n
            b[2] += "mgemm_kernel" in n or "dgemm_kernel" in n
    print("second: kernels / icache flushes / decode GEMMs")
    print("  " + "  ".join(f"{k}:{v[0]}/{v[1]}/{v[2]}" for k, v in sorted(per.items())))
    if a.skip_tuning:
        tune_end = max((e for s_, e_, n in rows if "flush_icache" in n and s_ <= hi for e in (e_,)), default=0)
        if tune_end < hi - 1e9:
            lo = max(lo, tune_end)
    if a.last_s > 0:
        lo = max(lo, hi - int(a.last_s * 1e9))
    lo, hi = lo + int(a.trim_s * 1e9), hi - int(a.trim_s * 1e9)
    win = [r for r in rows if lo <= r[0] and r[1] <= hi]
    if not win:
        print("empty window")
        return
    wall = hi - lo
    busy, cur_s, cur_e = 0, win[0][0], win[0][1]
    gaps, prev = [], win[0][2]
    agg = defaultdict(lambda: [0, 0])
    for s, e, n in win:
        agg[n][0] += e - s
        agg[n][1] += 1
    for s, e, n in win[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev, n))
            cur_s = s
        cur_e = max(cur_e, e)
        prev = n
    busy += cur_e - cur_s
    print(f"loaded span {wall / 1e9:.2f} s (trimmed {a.trim_s} s per end): GPU busy {100 * busy / wall:.1f} %, "
          f"{len(win)} kernels")
    big = [g for g in gaps if g[0] >= a.min_gap_us * 1e3]
    print(f"idle {(wall - busy) / 1e6:.1f} ms in {len(gaps)} gaps; gaps >= {a.min_gap_us:.0f} us: {len(big)}, "
          f"{sum(g[0] for g in big) / 1e6:.1f} ms")
    pairs = Counter()
    for d, p, n in big:
        pairs[(p[:60], n[:60])] += d
    for (p, n), d in pairs.most_common(8):
        print(f"  {d / 1e6:8.1f} ms  after {p}  before {n}")
    pre = ("pgemm", "flash_prefill_kernel<128, true", "rmsnorm_kernel<8", "rope_cache_kernel<false")
    tp = sum(t for k, (t, c) in agg.items() if any(x in k for x in pre))
    tot = sum(t for t, c in agg.values())
    print(f"kernel time: prefill-like {tp / 1e6:.1f} ms, the rest (decode, embed, search) {(tot - tp) / 1e6:.1f} ms")
    for k, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[: a.top]:
        print(f"{t / 1e6:9.1f} ms {c:8d} calls {t / max(1, c) / 1e3:8.1f} us/call  {k[:110]}")


if __name__ == "__main__":
    main()
