"""Block-sharing statistics of the bench's RAG decode batches (CPU, no GPU needed).

Rebuilds the bench's prompts (MiniLM random-init retrieval over the synthetic corpus, the
same chat template) and simulates the prefix cache at block granularity: two rows share a
KV block iff their prompts agree on every token up to the end of that block.  Reports the
cascade prefix (blocks shared by every row), the blocks each row reads beyond it, and the
K/V tile volume the grouped decode kernel streams per layer for the host's group packing
(ops.pack_decode_groups) vs. the ideal (every distinct block once).

    python scripts/group_stats.py [--batch 256] [--batches 3] [--max-new-tokens 128]
"""
from __future__ import annotations

import argparse
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--batches", type=int, default=3)
    ap.add_argument("--max-new-tokens", type=int, default=128)
    ap.add_argument("--notes", type=int, default=1000)
    ap.add_argument("--questions", choices=("unique", "repeat"), default="unique")
    a = ap.parse_args()

    import torch

    from docqa_amd import ops
    from docqa_amd.index.flat import FlatIndex
    from docqa_amd.models import checkpoint as ck
    from docqa_amd.pipeline.corpus import build_corpus, embed_records
    from docqa_amd.pipeline.rag import RAGPipeline
    from docqa_amd.text.synthetic import synthetic_questions, synthetic_unique_questions
    from docqa_amd.text.tokenizer import ChatTokenizer, WordPieceTokenizer

    torch.set_grad_enabled(False)
    llm_cfg = ck.resolve_llama_config("llama3-8b")
    enc_tok = WordPieceTokenizer()
    chat_tok = ChatTokenizer(model_vocab=llm_cfg.vocab_size)
    encoder = ck.resolve_bert("minilm-l6", device="cpu", seed=0)
    records = build_corpus(a.notes, None, 0)
    emb = embed_records(encoder, enc_tok, records)
    index = FlatIndex(encoder.cfg.hidden, "l2", "cpu", torch.float32, capacity=max(1024, len(records)))
    index.add(emb)

    class _Eng:
        device = torch.device("cpu")

    pipe = RAGPipeline(encoder, enc_tok, index, records, _Eng(), chat_tok, k=3, max_prompt_tokens=2048 - 256)
    gen = synthetic_unique_questions if a.questions == "unique" else synthetic_questions
    qs = gen((a.batches + 2) * a.batch, seed=123)
    BS = 64
    for bi in range(2, 2 + a.batches):   # the bench's timed batches follow 2 warm-up batches
        qb = qs[bi * a.batch:(bi + 1) * a.batch]
        _, I = pipe.retrieve(qb)
        prompts = pipe.build_prompts(qb, I.tolist())
        # physical block ids: one id per distinct full-block prefix; partial tail blocks private
        ids: dict[tuple, int] = {}
        tables, lens = [], []
        for r, p in enumerate(prompts):
            L = len(p) + a.max_new_tokens
            nb = (L + BS - 1) // BS
            tb = []
            for j in range(nb):
                if (j + 1) * BS <= len(p):
                    key = tuple(p[:(j + 1) * BS])
                else:
                    key = ("row", r, j)
                tb.append(ids.setdefault(key, len(ids)))
            tables.append(tb)
            lens.append(L)
        skip = 0
        while all(len(t) > skip and t[skip] == tables[0][skip] for t in tables) and (skip + 1) * BS <= min(map(len, prompts)):
            skip += 1
        per_row = [len(t) - skip for t in tables]
        distinct = len({b for t in tables for b in t[skip:]})
        quads = ops.pack_decode_groups(tables, lens, skip, BS, a.batch // 2)
        # half-block (32-token) tiles streamed by the group kernel at the END of decode
        def tiles(qd):
            seen = set()
            n = 0
            for r in qd:
                for pos in range(skip, len(tables[r])):
                    b = tables[r][pos]
                    if b in seen:
                        continue
                    seen.add(b)
                    live = [lens[x] for x in qd if len(tables[x]) > pos and tables[x][pos] == b]
                    n += 1 + (max(live) > pos * BS + 32)
            return n
        tl = [tiles(q) for q in quads]
        print(f"batch {bi}: prompt tokens mean {statistics.mean(map(len, prompts)):.0f} "
              f"min {min(map(len, prompts))} max {max(map(len, prompts))}; cascade prefix {skip} blocks")
        print(f"  blocks/row beyond prefix: mean {statistics.mean(per_row):.1f}; rows x blocks {sum(per_row)}, "
              f"distinct {distinct} (ideal sharing x{sum(per_row) / distinct:.2f})")
        print(f"  groups {len(quads)}: tiles/group mean {statistics.mean(tl):.1f} max {max(tl)} min {min(tl)}; "
              f"total tiles {sum(tl)} vs ideal {2 * distinct} -> per layer "
              f"{sum(tl) * 8 * 16 / 1024:.0f} MB (ideal {2 * distinct * 8 * 16 / 1024:.0f} MB)")
        # how many rows share each distinct block
        cnt: dict[int, int] = {}
        for t in tables:
            for b in t[skip:]:
                cnt[b] = cnt.get(b, 0) + 1
        hist: dict[int, int] = {}
        for c in cnt.values():
            k = 1 if c == 1 else 2 if c == 2 else 4 if c <= 4 else 8 if c <= 8 else 16 if c <= 16 else 99
            hist[k] = hist.get(k, 0) + 1
        print("  sharers per distinct block (<=):", dict(sorted(hist.items())))


if __name__ == "__main__":
    main()
