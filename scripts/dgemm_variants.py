"""Build dgemm.hip variants (-DDGV=n) on the GPU box and check each for wrong results."""
import ctypes
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch

CS = ROOT / "docqa_amd" / "csrc"
OUT = ROOT / "gpurun_out"
wrap = OUT / "dgv_wrap.hip"
wrap.write_text('#include "kernels/dgemm.hip"\nextern "C" int dg(const void* x, const void* w, void* y, float* p, int M, int N, int K, int S) {\n'
                '  return docqa_dgemm(x, w, y, p, M, N, K, S, 0); }\n')
torch.manual_seed(0)
N, K = 28672, 4096
w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
for v in [int(a) for a in sys.argv[1:]]:
    so = OUT / f"dgv_{v}.so"
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC", f"-I{CS/'include'}",
                    f"-I{CS}", f"-DDGV={v}", str(wrap), "-o", str(so)], check=True)
    lib = ctypes.CDLL(str(so))
    res = []
    for M in (1, 16, 64):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        ref = x.float() @ w.float().T
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        worst = 0.0
        for rep in range(10):
            y.zero_()
            torch.cuda.synchronize()
            rc = lib.dg(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(w.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                        None, M, N, K, 1)
            torch.cuda.synchronize()
            assert rc == 0
            worst = max(worst, (y.float() - ref).abs().max().item())
        res.append((M, round(worst, 3)))
        if v == 9:
            break
    # timing: gate_up M=1 / M=64 (S=1), rotating 5 weight copies past the MALL
    ws = [w] + [torch.randn_like(w) for _ in range(4)] if v == int(sys.argv[1]) else ws
    tm = []
    for M in (1, 64):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for it in range(25):
            if it == 5:
                s.record()
            lib.dg(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(ws[it % 5].data_ptr()), ctypes.c_void_p(y.data_ptr()),
                   None, M, N, K, 1)
        e.record()
        torch.cuda.synchronize()
        tm.append(round(s.elapsed_time(e) / 20 * 1e3, 1))
    print("variant", v, res, "us(M=1,64)", tm, flush=True)
