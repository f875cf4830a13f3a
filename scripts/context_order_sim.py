"""Prefix-cache hit rate of the bench workload per retrieved-context order, simulated on
the CPU (no generator): the bench's corpus, encoder, index and questions, the pipeline's
own prompt assembly, and a trie of 64-token blocks standing in for the engine's prefix
cache (blocks of earlier prompts -- same batch or earlier -- count as cached).
Usage: python scripts/context_order_sim.py [batches] [batch]"""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
os.environ.setdefault("QA_TEMPLATE", "cache_friendly")
import torch  # noqa: E402

from docqa_amd.index.flat import FlatIndex  # noqa: E402
from docqa_amd.models import checkpoint as ck  # noqa: E402
from docqa_amd.pipeline.corpus import build_corpus, embed_records  # noqa: E402
from docqa_amd.pipeline.rag import RAGPipeline  # noqa: E402
from docqa_amd.text.synthetic import synthetic_unique_questions  # noqa: E402
from docqa_amd.text.tokenizer import ChatTokenizer, WordPieceTokenizer  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 7
bs = int(sys.argv[2]) if len(sys.argv) > 2 else 256
torch.set_num_threads(8)
cfg = ck.resolve_llama_config("llama3-8b")
enc_tok, chat_tok = WordPieceTokenizer(), ChatTokenizer(model_vocab=cfg.vocab_size)
enc = ck.resolve_bert("minilm-l6", device="cpu", seed=0)
recs = build_corpus(1000, None, 0)
idx = FlatIndex(enc.cfg.hidden, "l2", "cpu", torch.float32, capacity=max(1024, len(recs)))
idx.add(embed_records(enc, enc_tok, recs))
qs = synthetic_unique_questions(nb * bs, seed=123)
res = {}
for order in (sys.argv[3].split(",") if len(sys.argv) > 3 else ("relevance", "shared", "trie")):
    pipe = RAGPipeline(enc, enc_tok, idx, recs, None, chat_tok, k=3, max_prompt_tokens=2048 - 256,
                       context_order=order)
    trie, tot, hit = set(), 0, 0
    per = []
    for b in range(nb):
        batch = qs[b * bs:(b + 1) * bs]
        _, I = pipe.retrieve(batch)
        prompts = pipe.build_prompts(batch, I.tolist())
        bt, bh = 0, 0
        for p in prompts:
            key = ()
            run = True
            for j in range(len(p) // 64):
                key = hash((key, tuple(p[64 * j:64 * j + 64])))
                if run and key in trie:
                    bh += 64
                else:
                    run = False
                    trie.add(key)
            bt += len(p)
        per.append(round(bh / bt, 3))
        tot += bt
        hit += bh
    res[order] = {"cached_frac_all": round(hit / tot, 3), "per_batch": per, "avg_prompt_tokens": round(tot / (nb * bs), 1)}
    print(order, res[order], flush=True)
