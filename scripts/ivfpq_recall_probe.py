"""Why IVF-PQ recall is low on the indexer's bge vectors, and what raises it (GPU probe).

Embeds synthetic clinical-note chunks with the bge-base encoder (random-init, HIP encoder
kernels) as the semantic indexer does, then builds IVF-PQ variants over the SAME vectors
and reports recall@10 against exact search: PQ sub-quantizer count M, and an orthogonal
pre-rotation of the space (exact for L2) -- a random rotation, and a PCA rotation whose
dimensions are dealt to the sub-quantizers round-robin so each gets an equal share of the
variance (random-init embeddings are strongly anisotropic: a few directions hold most of
the variance and land in a handful of sub-spaces).

    python scripts/ivfpq_recall_probe.py [--n 200000] [--nlist 1024]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200_000)
    ap.add_argument("--nlist", type=int, default=1024)
    ap.add_argument("--nq", type=int, default=256)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--variants", default="base64,base96,base128,rr64,pca64,pca96")
    a = ap.parse_args()

    from docqa_amd import ops
    from docqa_amd.index.ivfpq import IVFPQIndex
    from docqa_amd.models.bert import BertConfig, BertEncoder
    from docqa_amd.text.chunking import chunk_chars
    from docqa_amd.text.synthetic import synthetic_note, synthetic_unique_questions
    from docqa_amd.text.tokenizer import WordPieceTokenizer

    assert ops.load_native()
    torch.set_grad_enabled(False)
    enc = BertEncoder(BertConfig.preset("bge-base"), device="cuda")
    tok = WordPieceTokenizer(max_len=512)
    t = time.perf_counter()
    texts, i = [], 0
    while len(texts) < a.n:
        texts += chunk_chars(synthetic_note(i, seed=17)["text"], 500)
        i += 1
    texts = texts[: a.n]
    xb = torch.cat([enc.encode(tok.encode_batch(texts[j:j + 8192])).float() for j in range(0, a.n, 8192)])
    xq = enc.encode(tok.encode_batch(synthetic_unique_questions(a.nq, seed=5))).float()
    torch.cuda.synchronize()
    print(json.dumps({"embedded": a.n, "s": round(time.perf_counter() - t, 1)}), flush=True)

    def exact(x, q, k):
        d = (x * x).sum(1)[None] - 2 * q @ x.t()
        return torch.topk(d, k, dim=1, largest=False).indices

    gt = exact(xb, xq, a.k)
    mu = xb.mean(0)
    cov = torch.cov((xb - mu).t().double())
    ev, vec = torch.linalg.eigh(cov)                      # ascending
    ev, vec = ev.flip(0), vec.flip(1)
    top = (ev[:8] / ev.sum()).tolist()
    print(json.dumps({"variance_top8_frac": [round(v, 4) for v in top],
                      "variance_top64_frac": round(float(ev[:64].sum() / ev.sum()), 4)}), flush=True)

    def rotation(kind: str, M: int):
        if kind == "rr":
            g = torch.Generator(device="cpu").manual_seed(0)
            q, _ = torch.linalg.qr(torch.randn(xb.shape[1], xb.shape[1], generator=g, dtype=torch.float64))
            return q.float().cuda()
        if kind == "pca":
            d = xb.shape[1]
            # PCA dim r -> sub-space r % M: every sub-space gets every M-th eigen-direction
            order = torch.tensor([r for j in range(M) for r in range(j, d, M)])
            return vec[:, order].float().cuda()
        return None

    for v in a.variants.split(","):
        kind = "".join(c for c in v if c.isalpha())
        M = int("".join(c for c in v if c.isdigit()))
        R = rotation(kind, M)
        x = xb @ R if R is not None else xb
        q = xq @ R if R is not None else xq
        t = time.perf_counter()
        idx = IVFPQIndex(xb.shape[1], a.nlist, M, device="cuda")
        idx.train(x[: min(a.n, 100 * a.nlist)])
        idx.add(x)
        torch.cuda.synchronize()
        build = time.perf_counter() - t
        res = {"variant": v, "M": M, "rotation": kind, "build_s": round(build, 1)}
        for nprobe in (16, 32, 64):
            for kc in (a.k, 64):
                _, I = idx.search(q, kc, nprobe=nprobe)
                if kc > a.k:   # exact refine of the PQ candidates (as RefineFlat)
                    rows = x[I.clamp_min(0)]
                    dd = ((rows - q[:, None]) ** 2).sum(-1).masked_fill(I < 0, float("inf"))
                    I = torch.gather(I, 1, torch.topk(dd, a.k, dim=1, largest=False).indices)
                hit = sum(len(set(I[j].tolist()) & set(gt[j].tolist())) for j in range(a.nq))
                res[f"np{nprobe}_c{kc}"] = round(hit / (a.nq * a.k), 4)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
