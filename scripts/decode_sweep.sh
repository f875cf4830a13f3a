#!/bin/bash
# sweep the decode split target on the kernel micro-benchmark (one process per setting)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for t in ${SWEEP_TARGETS:-512}; do
  DOCQA_DECODE_WG_TARGET=$t timeout -k 10 300 python -c "
import json, math, torch, sys
sys.path.insert(0, '.')
from benchmarks.bench_kernels import timeit
from docqa_amd import ops
ops.load_native(); nat = torch.ops.docqa
res = []
for (B, ctx) in [(64, 640), (64, 1024), (1, 4096), (8, 1024), (256, 1024)]:
    Hq, Hkv, D, BS = 32, 8, 128, 64
    maxb = (ctx + BS - 1) // BS
    kc = torch.randn(B * maxb, Hkv, BS, D, device='cuda', dtype=torch.bfloat16); vc = torch.randn_like(kc)
    bt = torch.arange(B * maxb, device='cuda', dtype=torch.int32).view(B, maxb)
    cl = torch.full((B,), ctx, device='cuda', dtype=torch.int32)
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device='cuda', dtype=torch.bfloat16)
    t = timeit(lambda: nat.paged_decode(q, kc, vc, bt, cl, Hq, 2048 if ctx < 2048 else 4096, 1 / math.sqrt(D)))
    res.append((B, ctx, round(t, 1), round(2 * B * ctx * Hkv * D * 2 / t / 1e6, 2)))
print('target', $t, res)
" >> gpurun_out/decode_sweep.log 2>&1 || exit $?
done
