"""Run one mid-M decode GEMM shape repeatedly (weights rotated past the MALL) for PMC
counter collection: rocprofv3 --pmc <counters> -- python scripts/mgemm_pmc_probe.py
{mgemm|glu|wgemm|wglu|argmax|hipblaslt} M N K S bn"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import torch.nn.functional as F

from docqa_amd import ops


def main():
    op = sys.argv[1]
    M, N, K, S, bn = (int(v) for v in sys.argv[2:7])
    assert ops.load_native()
    nat = torch.ops.docqa
    nb = N * K * 2
    copies = max(2, (1 << 30) // nb + 1)
    ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(copies)]
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    mt = (M + 255) // 256
    wsb = torch.empty(mt * N * 256, device="cuda", dtype=torch.float32)
    tick = torch.zeros(2 * mt * N // 128 + 1, device="cuda", dtype=torch.int32)
    fn = {"mgemm": lambda w: nat.mgemm(x, w, S, bn), "glu": lambda w: nat.mgemm_glu(x, w, bn),
          "wgemm": lambda w: nat.wgemm(x, w, S, bn), "wglu": lambda w: nat.wgemm_glu(x, w, S, bn, wsb, tick),
          "argmax": lambda w: nat.mgemm_argmax(x, w, N, bn), "hipblaslt": lambda w: F.linear(x, w)}[op]
    for i in range(4 * copies):
        fn(ws[i % copies])
    torch.cuda.synchronize()
    print("done", op, M, N, K, S, bn, copies)


if __name__ == "__main__":
    main()
