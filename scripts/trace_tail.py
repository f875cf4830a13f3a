"""Summarise the tail of a rocprofv3 kernel trace: per-kernel time over the last
``--window-ms`` of GPU activity (e.g. the timed decode iteration of gen_probe.py, after
TunableOp tuning and warm-up have polluted the whole-run --stats table).

Usage: python scripts/trace_tail.py <run_kernel_trace.csv> --window-ms 690 [--steps 63]
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window-ms", type=float, required=True)
    ap.add_argument("--steps", type=int, default=1, help="divide totals by this (per-step view)")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--gaps", type=int, default=0, help="also list the N largest idle gaps in the window")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    end = max(e for _, e, _ in rows)
    t0 = end - int(a.window_ms * 1e6)
    agg = defaultdict(lambda: [0, 0])
    busy = 0
    for s, e, n in rows:
        if s >= t0:
            agg[n][0] += e - s
            agg[n][1] += 1
            busy += e - s
    print(f"window {a.window_ms} ms: kernel-busy {busy/1e6:.2f} ms, per step {busy/1e3/a.steps:.1f} us")
    for n, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[: a.top]:
        print(f"{t/1e3/a.steps:9.1f} us/step {c/a.steps:7.1f} calls/step {t/max(1,c)/1e3:8.1f} us/call  {n[:120]}")
    if a.gaps:
        win = sorted((s, e, n) for s, e, n in rows if s >= t0)
        gaps, cur_end, prev = [], win[0][1], win[0][2]
        for s, e, n in win[1:]:
            if s > cur_end:
                gaps.append((s - cur_end, prev, n))
            if e > cur_end:
                cur_end, prev = e, n
        idle = sum(g for g, _, _ in gaps)
        print(f"idle (no kernel running) {idle/1e6:.2f} ms in {len(gaps)} gaps; "
              f"gaps > 50 us: {sum(g for g, _, _ in gaps if g > 50000)/1e6:.2f} ms")
        for g, p, n in sorted(gaps, reverse=True)[: a.gaps]:
            print(f"  gap {g/1e3:9.1f} us  after {p[:60]}  before {n[:60]}")


if __name__ == "__main__":
    main()
