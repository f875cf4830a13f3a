"""Clock / power samples while a workload runs: is the decode step clock-limited?

Runs the given command (default: the headline bench) as a child process and samples
``rocm-smi -P -c --json`` every ~0.3 s until it exits; prints one JSON summary line (the
socket power and shader clock over the samples taken while the child ran, plus the power
cap) and writes every sample to gpurun_out/power_samples.jsonl.  The parent never touches
the GPU runtime (rocm-smi reads the driver's sysfs counters).

Usage: python scripts/power_probe.py [command ...]
"""
import json
import re
import statistics
import subprocess
import sys
import time
from pathlib import Path


def smi(*args):
    try:
        out = subprocess.run(["rocm-smi", *args, "--json"], capture_output=True, text=True, timeout=20).stdout
        return json.loads(out or "{}")
    except Exception as e:  # noqa: BLE001 -- a sample that fails is skipped, not fatal
        return {"error": str(e)}


def num(v):
    m = re.search(r"[-+]?\d+(\.\d+)?", str(v))
    return float(m.group(0)) if m else None


def main():
    cmd = sys.argv[1:] or [sys.executable, "bench.py", "--steps", "10", "--warmup", "2"]
    Path("gpurun_out").mkdir(exist_ok=True)
    cap = smi("--showmaxpower")
    child = subprocess.Popen(cmd)
    t0 = time.time()
    samples = []
    with open("gpurun_out/power_samples.jsonl", "w") as f:
        while child.poll() is None:
            s = smi("-P", "-c")
            s["t"] = round(time.time() - t0, 2)
            samples.append(s)
            f.write(json.dumps(s) + "\n")
            f.flush()
            time.sleep(0.3)
    rc = child.wait()
    power, sclk = [], []
    for s in samples:
        for card, d in s.items():
            if not isinstance(d, dict):
                continue
            for k, v in d.items():
                kl = k.lower()
                if "power" in kl and "(w)" in kl:
                    x = num(v)
                    if x:
                        power.append(x)
                if kl.startswith("sclk") and "clock" in kl:
                    x = num(v)
                    if x:
                        sclk.append(x)

    def q(xs):
        if not xs:
            return None
        xs = sorted(xs)
        return {"n": len(xs), "p10": xs[len(xs) // 10], "p50": statistics.median(xs), "p90": xs[9 * len(xs) // 10],
                "max": xs[-1]}
    print(json.dumps({"cmd": " ".join(cmd), "rc": rc, "secs": round(time.time() - t0, 1), "power_W": q(power),
                      "sclk_MHz": q(sclk), "cap": cap}), flush=True)
    sys.exit(rc)


if __name__ == "__main__":
    main()
