"""Run one decode-GEMM shape repeatedly (weights rotated past the MALL) for PMC counter
collection: rocprofv3 --pmc <counters> -- python scripts/dgemm_pmc_probe.py M N K S tile."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

from docqa_amd import ops


def main():
    M, N, K, S, tile = (int(v) for v in sys.argv[1:6])
    assert ops.load_native()
    nat = torch.ops.docqa
    nb = N * K * 2
    copies = max(2, (1 << 30) // nb + 1)
    ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(copies)]
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    for i in range(4 * copies):
        nat.dgemm_partial(x, ws[i % copies], S, tile)
    torch.cuda.synchronize()
    print("done", M, N, K, S, tile, copies)


if __name__ == "__main__":
    main()
