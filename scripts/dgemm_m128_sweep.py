"""Decode-GEMM sweep at 65-128 rows (Llama-3-8B projections): dgemm_partial over split
counts / tile widths and dgemm_glu vs hipBLASLt, weights rotated past the MALL.
Correctness of every timed variant is checked against an fp32 GEMM first."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
import torch.nn.functional as F

from benchmarks.bench_kernels import timeit
from docqa_amd import ops


def main():
    assert ops.load_native()
    nat = torch.ops.docqa
    Ms = [int(m) for m in (sys.argv[1].split(",") if len(sys.argv) > 1 and sys.argv[1][0].isdigit() else ["64", "96", "128"])]
    projs = [("qkv", 6144, 4096), ("o", 4096, 4096), ("down", 4096, 14336), ("gate_up", 28672, 4096)]
    if "--lm-head" in sys.argv:
        projs = [("lm_head", 128256, 4096)]
    for (name, N, K) in projs:
        nb = N * K * 2
        copies = max(2, (1 << 30) // nb + 1)
        ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(copies)]
        for M in Ms:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            ref = x.float() @ ws[0].float().T
            it = iter(range(1 << 30))
            row = {"proj": name, "M": M}
            row["hipblaslt_us"] = round(timeit(lambda: F.linear(x, ws[next(it) % copies]), iters=4 * copies), 1)
            if name == "gate_up" and M > 128:
                pass
            elif name == "gate_up":
                y = nat.dgemm_glu(x, ws[0])
                gu = ref.bfloat16()
                from docqa_amd.ops import reference as R
                err = (y.float() - R.silu_mul(gu, interleaved=True).float()).abs().max().item()
                row["glu_err"] = round(err, 4)
                row["glu_us"] = round(timeit(lambda: nat.dgemm_glu(x, ws[next(it) % copies]), iters=4 * copies), 1)
                row["hipblaslt_silu_us"] = round(timeit(lambda: nat.silu_mul(F.linear(x, ws[next(it) % copies]), True),
                                                        iters=4 * copies), 1)
            else:
                for tr in (64, 128):
                    for S in ((1,) if name == "lm_head" else (1, 2, 4, 7, 8)):
                        if K % S or (K // S) % 512 or N % tr :
                            continue
                        P = nat.dgemm_partial(x, ws[0], S, tr)
                        err = (P.sum(0) - ref).abs().max().item()
                        assert err < 0.1, (name, M, S, tr, err)
                        t = timeit(lambda: nat.dgemm_partial(x, ws[next(it) % copies], S, tr), iters=4 * copies)
                        row[f"S{S}_t{tr}_us"] = round(t, 1)
            print(json.dumps(row), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
