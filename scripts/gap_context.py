"""Host markers (ROCTX ranges, rocprofv3 --marker-trace) around the largest GPU-idle gaps
of a kernel trace: what the host was doing while the GPU had nothing queued.
Usage: python scripts/gap_context.py <run_kernel_trace.csv> <run_marker_api_trace.csv> [--gaps 3]"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernels")
    ap.add_argument("markers")
    ap.add_argument("--gaps", type=int, default=3)
    ap.add_argument("--min-us", type=float, default=1000)
    ap.add_argument("--window-ms", type=float, default=0, help="only the last N ms of GPU activity")
    a = ap.parse_args()
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 f'{r["Kernel_Name"][:50]} [q{r.get("Queue_Id", "?")} s{r.get("Stream_Id", "?")} t{r.get("Thread_Id", "?")}]')
                for r in csv.DictReader(open(a.kernels)))
    if a.window_ms:
        last = max(e for _, e, _ in ks)
        ks = [k for k in ks if k[0] >= last - a.window_ms * 1e6]
    ms = []
    for r in csv.DictReader(open(a.markers)):
        name = r.get("Function") or r.get("Operation") or r.get("Name") or "?"
        msg = r.get("Message") or r.get("Marker_Message") or ""
        ms.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), f"{name} {msg}"[:70], r.get("Thread_Id", "")))
    ms.sort()
    gaps, end, prev = [], ks[0][1], ks[0][2]
    for s, e, n in ks[1:]:
        if s - end > a.min_us * 1e3:
            gaps.append((s - end, end, s, prev, n))
        if e > end:
            end, prev = e, n
    t0 = ks[0][0]
    for g, gs, ge, p, n in sorted(gaps, reverse=True)[: a.gaps]:
        print(f"gap {g/1e3:.1f} us at +{(gs - t0)/1e6:.1f} ms: after {p} before {n}")
        for s, e, m, tid in ms:
            if e >= gs - 20e6 and s <= ge + 2e6:
                print(f"    [{(s - gs)/1e3:+10.1f} .. {(e - gs)/1e3:+10.1f} us] tid {tid} {m}")


if __name__ == "__main__":
    main()
