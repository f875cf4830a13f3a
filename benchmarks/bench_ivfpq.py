"""BASELINE.json config 2: semantic-indexer bge-base-en embed + 10M-vector IVF-PQ kNN on
one MI355X.

Database: N synthetic 768-d vectors drawn from a Gaussian mixture (generating 10M real
bge embeddings offline would take the whole GPU budget; the search kernels only see
vectors).  Queries: synthetic clinical questions embedded by the bge-base encoder
(random-init weights) and mapped into the database distribution by adding a nearby
database vector (so every query has true neighbours), then searched with IVF-PQ and,
for recall, with the exact flat MFMA kernel over the same 10M vectors (30 GB fp32 in HBM).

Reports: build time (train + add), IVF-PQ search QPS at batch sizes, recall@10 vs exact,
embed throughput.  One JSON line.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--nlist", type=int, default=4096)
    ap.add_argument("--M", type=int, default=64)
    ap.add_argument("--nprobe", type=int, default=32)
    ap.add_argument("--nq", type=int, default=256)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()

    from docqa_amd import ops
    from docqa_amd.index.flat import FlatIndex
    from docqa_amd.index.ivfpq import IVFPQIndex
    from docqa_amd.models.bert import BertConfig, BertEncoder
    from docqa_amd.text.synthetic import synthetic_questions
    from docqa_amd.text.tokenizer import WordPieceTokenizer

    assert ops.load_native()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    ncent = 8192
    centers = torch.randn(ncent, a.d, device=dev, generator=g)
    xb = torch.empty(a.n, a.d, device=dev)
    chunk = 1 << 20
    for i in range(0, a.n, chunk):
        m = min(chunk, a.n - i)
        lab = torch.randint(0, ncent, (m,), device=dev, generator=g)
        xb[i:i + m] = centers[lab] + 0.5 * torch.randn(m, a.d, device=dev, generator=g)
    torch.cuda.synchronize()

    # queries: bge-base embeddings of clinical questions (+ a database anchor)
    enc = BertEncoder(BertConfig.preset("bge-base"), device=dev)
    tok = WordPieceTokenizer(max_len=512)
    qs = synthetic_questions(a.nq, seed=5)
    toks = tok.encode_batch(qs)
    enc.encode(toks[:8])
    torch.cuda.synchronize()
    t = time.perf_counter()
    qe = enc.encode(toks)
    torch.cuda.synchronize()
    embed_s = time.perf_counter() - t
    anchor = xb[torch.randint(0, a.n, (a.nq,), device=dev, generator=g)]
    xq = (anchor + 0.3 * qe * (a.d ** 0.5) * 0.05).contiguous()

    t = time.perf_counter()
    idx = IVFPQIndex(a.d, a.nlist, a.M, device=dev)
    idx.train(xb, niter=10)
    torch.cuda.synchronize()
    train_s = time.perf_counter() - t
    t = time.perf_counter()
    idx.add(xb)
    torch.cuda.synchronize()
    add_s = time.perf_counter() - t

    res = {}
    for bs in (1, 16, 256):
        q = xq[:bs]
        idx.search(q, a.k, a.nprobe)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            D, I = idx.search(q, a.k, a.nprobe)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.iters
        res[f"batch{bs}"] = {"ms": round(dt * 1e3, 3), "qps": round(bs / dt, 1)}

    flat = FlatIndex(a.d, "l2", dev, capacity=1)
    flat._xb, flat._norms, flat.ntotal = xb, (xb ** 2).sum(1), a.n
    torch.cuda.synchronize()
    t = time.perf_counter()
    De, Ie = flat.search(xq, a.k)
    torch.cuda.synchronize()
    flat_s = time.perf_counter() - t
    _, Ia = idx.search(xq, a.k, a.nprobe)
    recall = sum(len(set(Ia[i].tolist()) & set(Ie[i].tolist())) for i in range(a.nq)) / (a.nq * a.k)
    r1 = (Ia[:, 0] == Ie[:, 0]).float().mean().item()
    out = {"metric": "ivfpq_search_qps", "config": f"IVF{a.nlist},PQ{a.M} n={a.n} d={a.d} nprobe={a.nprobe} k={a.k}",
           "search": res, "recall_at_k": round(recall, 4), "recall_1_at_1": round(r1, 4),
           "train_s": round(train_s, 2), "add_s": round(add_s, 2),
           "exact_flat_ms_per_batch": round(flat_s * 1e3, 2), "exact_flat_batch": a.nq,
           "bge_embed_qps": round(a.nq / embed_s, 1), "codes_bytes": idx.codes.numel()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
