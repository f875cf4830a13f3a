"""Race detection / sanitizers for the native host runtime: the KV
block manager core (csrc/runtime/block_manager_core.h) -- the structure the scheduler
thread, the QA batcher and the engine share -- is built into a multi-threaded stress test
under ThreadSanitizer and under AddressSanitizer + UndefinedBehaviorSanitizer and run on
the CPU.  Any report fails the test (sanitizers exit non-zero)."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "docqa_amd" / "csrc" / "tests" / "block_manager_stress.cpp"


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_block_manager_under_sanitizer(tmp_path, san):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = tmp_path / f"bm_{san.replace(',', '_')}"
    r = subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={san}",
                        "-fno-sanitize-recover=all", "-pthread", str(SRC), "-o", str(exe)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    run = subprocess.run([str(exe), "8", "1500", "24"], capture_output=True, text=True, timeout=600, env=env)
    assert run.returncode == 0 and "OK" in run.stdout, (run.stdout + run.stderr)[-4000:]
    # exhaustion is exercised deterministically at the end of the program (the threaded
    # phase reaches it only when the scheduler overlaps enough threads -- not on a loaded box)
