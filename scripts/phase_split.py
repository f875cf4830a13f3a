"""Per-batch phase split of a rocprofv3 kernel trace of bench.py: for each 256-question
batch, the wall span and the kernel-busy time of its prefill (first prefill GEMM ->
first decode attention launch) and of its decode loop, and the GPU gap between batches.
Kernel-busy < wall inside a phase means the GPU waited on the host there.

Usage: python scripts/phase_split.py <run_kernel_trace.csv> [--last N] [--kernels]
(--kernels: per-kernel calls / busy ms / share inside the last batch's prefill phase)
"""
import argparse
import csv


def kind(name: str) -> str:
    if "pgemm_kernel" in name or name.startswith("void (anonymous namespace)::gemm_kernel"):
        return "P"
    if "paged_decode" in name or "mgemm_kernel" in name:
        return "D"
    return "-"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=4)
    ap.add_argument("--kernels", action="store_true")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # batch starts: a prefill kernel after at least one decode kernel (or the first one)
    starts, seen_decode = [], True
    for i, (s, e, n) in enumerate(rows):
        k = kind(n)
        if k == "P" and seen_decode:
            starts.append(i)
            seen_decode = False
        elif k == "D":
            seen_decode = True
    out, pres = [], []
    for bi, si in enumerate(starts):
        ei = starts[bi + 1] if bi + 1 < len(starts) else len(rows)
        seg = rows[si:ei]
        d0 = next((j for j, r in enumerate(seg) if "paged_decode" in r[2]), None)
        if d0 is None:
            continue
        # prefill phase = kernels before the first decode attention minus the decode-graph
        # preamble; decode = the rest up to the last decode-kind kernel
        dl = max(j for j, r in enumerate(seg) if kind(r[2]) == "D")
        pre, dec = seg[:d0], seg[d0:dl + 1]
        pres.append(pre)

        def busy(xs):
            return sum(e - s for s, e, _ in xs) / 1e6

        p_wall = (seg[d0][0] - seg[0][0]) / 1e6
        d_wall = (dec[-1][1] - dec[0][0]) / 1e6
        gap = ((rows[ei][0] - dec[-1][1]) / 1e6) if ei < len(rows) else None
        out.append({"prefill_wall_ms": round(p_wall, 2), "prefill_busy_ms": round(busy(pre), 2),
                    "decode_wall_ms": round(d_wall, 2), "decode_busy_ms": round(busy(dec), 2),
                    "decode_kernels": len(dec), "gap_to_next_batch_ms": None if gap is None else round(gap, 2)})
    for o in out[-a.last:]:
        print(o)
    # the longest prefill phase among the last N batches (a pipelined batch's prefill can be
    # queued behind the previous decode, which splits a short preamble off as its own phase)
    last_pre = max(pres[-a.last:], key=lambda p: sum(e - s for s, e, _ in p)) if pres else None
    if a.kernels and last_pre:
        tot = sum(e - s for s, e, _ in last_pre)
        agg = {}
        for s, e, n in last_pre:
            c = agg.setdefault(n[:120], [0, 0])
            c[0] += 1
            c[1] += e - s
        print(f"# longest recent prefill phase: {len(last_pre)} kernels, busy {tot / 1e6:.2f} ms")
        for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"{t / 1e6:9.2f} ms {c:6d} {100 * t / tot:5.1f}%  {n}")


if __name__ == "__main__":
    main()
