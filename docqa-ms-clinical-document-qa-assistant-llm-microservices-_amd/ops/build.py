"""In-tree build of the gfx950 HIP kernels + torch operator bindings.

Produces ``docqa_amd/ops/_docqa_C.so`` (git-ignored, but it travels with the repo
snapshot to the GPU box).  No JIT cache under ``~/.cache`` is used: the kernels are
compiled once, here, with ``hipcc --offload-arch=gfx950``.

Layout:
  csrc/kernels/*.hip   device code, no torch headers (fast to compile, seconds each)
  csrc/bindings.cpp    TORCH_LIBRARY registration (torch headers, compiled once)
  csrc/runtime/*.cpp   native host runtime (paged-KV block manager, scheduler, IO)

Run: ``python -m docqa_amd.ops.build`` (or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent.parent
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build" / "docqa"
OUT = PKG / "ops" / "_docqa_C.so"
ARCH = os.environ.get("DOCQA_OFFLOAD_ARCH", "gfx950")

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce

    root = Path(torch.__file__).resolve().parent
    incs = [str(root / "include"), str(root / "include" / "torch" / "csrc" / "api" / "include")]
    libdir = str(root / "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return incs, libdir, abi


def _hash_file(p: Path, extra: str = "") -> str:
    h = hashlib.sha1(p.read_bytes())
    for inc in sorted((CSRC / "include").glob("*.h")):
        h.update(inc.read_bytes())
    h.update(extra.encode())
    return h.hexdigest()[:16]


def _run(cmd, desc):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"[docqa build] {desc} failed:\n{' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def _compile(src: Path, flags: list[str], kind: str) -> Path:
    key = _hash_file(src, " ".join(flags))
    obj = BUILD / f"{src.stem}.{kind}.{key}.o"
    if obj.exists():
        return obj
    for stale in BUILD.glob(f"{src.stem}.{kind}.*.o"):
        stale.unlink()
    tmp = obj.with_suffix(".tmp.o")
    _run([HIPCC, *flags, "-c", str(src), "-o", str(tmp)], f"compile {src.name}")
    tmp.rename(obj)
    return obj


def build(verbose: bool = True, jobs: int | None = None) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    incs, libdir, abi = _torch_paths()
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{CSRC / 'include'}", f"-D_GLIBCXX_USE_CXX11_ABI={abi}"]
    dev_flags = common + [f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]
    host_flags = common + [
        "-x", "hip", f"--offload-arch={ARCH}",
        "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_docqa_C",
        f"-I{sysconfig.get_paths()['include']}",
        *[f"-I{i}" for i in incs], "-Wno-unused-result", "-Wno-deprecated-declarations",
    ]
    kernels = sorted((CSRC / "kernels").glob("*.hip"))
    runtime = sorted((CSRC / "runtime").glob("*.cpp"))
    jobs = jobs or min(16, os.cpu_count() or 4)
    objs: list[Path] = []
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile, k, dev_flags, "dev") for k in kernels]
        futs += [ex.submit(_compile, r, host_flags, "rt") for r in runtime]
        futs.append(ex.submit(_compile, CSRC / "bindings.cpp", host_flags, "bind"))
        for f in futs:
            objs.append(f.result())
    link_key = hashlib.sha1("".join(sorted(o.name for o in objs)).encode()).hexdigest()[:16]
    stamp = BUILD / "link.stamp"
    if OUT.exists() and stamp.exists() and stamp.read_text() == link_key:
        if verbose:
            print(f"[docqa build] up to date: {OUT}")
        return OUT
    tmp = OUT.with_suffix(".tmp.so")
    _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), f"-L{libdir}",
          "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
          f"-Wl,-rpath,{libdir}", "-o", str(tmp)], "link")
    tmp.rename(OUT)
    stamp.write_text(link_key)
    if verbose:
        print(f"[docqa build] built {OUT} from {len(objs)} objects")
    return OUT


if __name__ == "__main__":
    build()
    sys.exit(0)
