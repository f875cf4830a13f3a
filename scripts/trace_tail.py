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


if __name__ == "__main__":
    main()
