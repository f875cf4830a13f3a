"""Grouped vs per-row cascade decode attention on a RAG-like batch (common template prefix,
clusters of rows sharing prefix-cache blocks, unique tails), caches rotated past the MALL.
Usage: python scripts/group_decode_probe.py [B]"""
import json
import math
import os
import random
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

from benchmarks.bench_kernels import timeit
from docqa_amd import ops


def batch(B, Pb, maxb, seed=0):
    rnd = random.Random(seed)
    nxt = Pb
    tables, lens = [], []
    while len(tables) < B:
        csize = rnd.choices([1, 2, 3, 4, 6], [40, 25, 15, 12, 8])[0]
        depth = rnd.randint(2, 4)
        shared = list(range(nxt, nxt + depth))
        nxt += depth
        for _ in range(min(csize, B - len(tables))):
            own = list(range(nxt, nxt + maxb - Pb - depth))
            nxt += len(own)
            tables.append(list(range(Pb)) + shared + own)
            lens.append(64 * (Pb + depth) + rnd.randint(40, 250))
    return tables, lens, nxt


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    assert ops.load_native()
    Hkv, D, BS, Pb, maxb = 8, 128, 64, 5, 32
    Hq = 4 * Hkv
    tables, lens, nblk = batch(B, Pb, maxb)
    nb = 2 * nblk * Hkv * BS * D * 2
    copies = max(2, (1 << 30) // nb + 1)
    caches = [(torch.randn(nblk, Hkv, BS, D, device="cuda", dtype=torch.bfloat16),
               torch.randn(nblk, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)) for _ in range(copies)]
    bt = torch.tensor(tables, dtype=torch.int32, device="cuda")
    cl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    pt = bt[0].clone()
    plen = torch.tensor([Pb * BS], dtype=torch.int32, device="cuda")
    scale = 1 / math.sqrt(D)
    order = torch.argsort(cl.cpu(), descending=True).int().cuda()
    cap = (B + 1) // 2
    quads = ops.pack_decode_groups(tables, lens, Pb, BS, cap)
    flat = torch.full((cap * 4,), -1, dtype=torch.int32)
    for i, qd in enumerate(quads):
        flat[4 * i:4 * i + len(qd)] = torch.tensor(qd, dtype=torch.int32)
    groups = flat.cuda()
    nchunk = 8
    per_row = sum(len(t[Pb:(l + 63) // 64]) for t, l in zip(tables, lens))
    grouped = sum(len({b for r in qd for b in tables[r][Pb:(lens[r] + 63) // 64]}) for qd in quads)
    it = iter(range(1 << 30))
    t_ring = timeit(lambda: ops.paged_decode_cascade(q, *caches[next(it) % copies], bt, cl, Hq, maxb * BS, scale,
                                                      pt, plen, nchunk, order), iters=4 * copies)
    it = iter(range(1 << 30))
    t_grp = timeit(lambda: ops.paged_decode_cascade_grouped(q, *caches[next(it) % copies], bt, cl, Hq, scale, pt,
                                                            plen, nchunk, groups), iters=4 * copies)
    plan = ops.split_decode_groups(quads, tables, lens, Pb, BS, B, int(os.environ.get("DOCQA_GROUP_TILES", "12"))).cuda()
    it = iter(range(1 << 30))
    t_split = timeit(lambda: ops.paged_decode_cascade_grouped(q, *caches[next(it) % copies], bt, cl, Hq, scale, pt,
                                                              plen, nchunk, plan), iters=4 * copies)
    tiles = sum(t for qd in quads for _, t in ops.group_tiles_by_position(tables, lens, qd, Pb, BS))
    kv_row = 2 * sum(l - Pb * BS for l in lens) * Hkv * D * 2
    print(json.dumps({"B": B, "groups": len(quads), "per_row_blocks": per_row, "grouped_blocks": grouped,
                      "split_us": round(t_split, 1), "split_tiles_MB": round(tiles * Hkv * 16 / 1024, 1),
                      "split_TBps": round(tiles * Hkv * 16384 / t_split / 1e6, 2),
                      "ring_us": round(t_ring, 1), "grouped_us": round(t_grp, 1),
                      "ring_suffix_TBps": round(kv_row / t_ring / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
