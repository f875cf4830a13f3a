"""Print grid sizes / durations of every launch of kernels matching a pattern in a
rocprofv3 kernel trace (last --window-ms of activity)."""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("pattern")
    ap.add_argument("--window-ms", type=float, default=1e9)
    ap.add_argument("--limit", type=int, default=80)
    ap.add_argument("--from-ms", type=float, default=0.0, help="offset into the window")
    ap.add_argument("--to-ms", type=float, default=1e12)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    end = max(int(r["End_Timestamp"]) for r in rows)
    t0 = end - int(a.window_ms * 1e6)
    keys = [k for k in rows[0] if "Grid" in k or "Workgroup" in k or "LDS" in k or "VGPR" in k]
    n = 0
    for r in rows:
        rel = (int(r["Start_Timestamp"]) - t0) / 1e6
        if a.pattern in r["Kernel_Name"] and int(r["Start_Timestamp"]) >= t0 and a.from_ms <= rel <= a.to_ms:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            print(f"{(int(r['Start_Timestamp']) - t0) / 1e6:9.3f} ms  {d:9.1f} us  " +
                  " ".join(f"{k}={r[k]}" for k in keys) + f"  {r['Kernel_Name'][:60]}")
            n += 1
            if n >= a.limit:
                break


if __name__ == "__main__":
    main()
