import sys; sys.path.insert(0, "/root/repo")
import torch
from benchmarks.bench_kernels import timeit
from docqa_amd import ops
assert ops.load_native()
nat = torch.ops.docqa
N, K = 4096, 14336
copies = 10
ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16() for _ in range(copies)]
for M in (64, 128):
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    ref = x.float() @ ws[0].float().T
    for S, tr in [(4, 64), (7, 64), (14, 64), (7, 128), (14, 128)]:
        P = nat.dgemm_partial(x, ws[0], S, tr)
        assert (P.sum(0) - ref).abs().max().item() < 0.1
        it = iter(range(1 << 30))
        t = timeit(lambda: nat.dgemm_partial(x, ws[next(it) % copies], S, tr), iters=4 * copies)
        print(f"down M={M} S={S} tile={tr}: {t:.1f} us", flush=True)
