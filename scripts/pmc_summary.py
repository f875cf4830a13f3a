"""Per-kernel means of a rocprofv3 --pmc counter CSV (kernels whose name matches a
substring): python scripts/pmc_summary.py <dir-with-run_counter_collection.csv> <substr>..."""
import csv
import sys
from collections import defaultdict
from pathlib import Path


def summarize(path: Path, subs: list[str]) -> dict:
    per = defaultdict(lambda: defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if subs and not any(s in name for s in subs):
            continue
        key = name[:70]
        d = (r["Dispatch_Id"])
        per[key][("_n", d)] = 1
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        per[key][("_t", d)] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        meta[key] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"])
    out = {}
    for k, v in per.items():
        n = sum(1 for kk in v if isinstance(kk, tuple) and kk[0] == "_n")
        t = sum(val for kk, val in v.items() if isinstance(kk, tuple) and kk[0] == "_t") / n
        out[k] = {"dispatches": n, "mean_us": round(t, 1), "vgpr/agpr/lds": meta[k],
                  **{c: round(val / n) for c, val in v.items() if not isinstance(c, tuple)}}
    return out


if __name__ == "__main__":
    d = Path(sys.argv[1])
    for k, v in summarize(d / "run_counter_collection.csv", sys.argv[2:]).items():
        print(d.name, k, v)
