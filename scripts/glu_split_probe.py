import sys, json
sys.path.insert(0, '/root/repo')
import torch
from benchmarks.bench_kernels import timeit
from docqa_amd import ops
ops.load_native()
nat = torch.ops.docqa
N, K, M = 28672, 4096, 256
copies = 6
ws = [(torch.randn(N, K, device="cuda") / 64).bfloat16() for _ in range(copies)]
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
res = {}
for cfg, S in [(2, 1), (3, 2), (4, 2), (5, 2), (6, 2), (2, 2), (3, 1), (4, 1)]:
    it = iter(range(1 << 30))
    try:
        res[f"c{cfg}_S{S}"] = round(timeit(lambda: nat.mgemm(x, ws[next(it) % copies], S, cfg), iters=4 * copies), 1)
    except RuntimeError as e:
        res[f"c{cfg}_S{S}"] = str(e)[:40]
it = iter(range(1 << 30))
res["glu2"] = round(timeit(lambda: nat.mgemm_glu(x, ws[next(it) % copies], 2), iters=4 * copies), 1)
print(json.dumps(res))
