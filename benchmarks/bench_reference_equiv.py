"""Reference-equivalent QA serving on the same MI355X, to give the headline metric a
measured baseline (the reference publishes none -- BASELINE.md).

What the reference does per /ask/ request (llm-qa/main.py:111-122): one request at a
time (blocking ``qa_chain.invoke`` inside the handler, single uvicorn worker), MiniLM
query embedding (sentence-transformers, PyTorch eager), FAISS IndexFlatL2 k=3, LangChain
"stuff" prompt, and a greedy generation of a 7-8B decoder by a generic runtime (Ollama /
llama.cpp).  Its public GPU equivalent here: PyTorch eager MiniLM (HF ``BertModel``),
exact L2 search in PyTorch, and Hugging Face ``LlamaForCausalLM.generate`` (greedy,
KV cache, SDPA attention, bf16, batch 1) for Llama-3-8B -- same model architecture, same
prompt lengths, same number of new tokens as ``bench.py``, random-init weights.

Output: one JSON line with queries/s and p50 latency of that serial loop.
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", type=int, default=8)
    ap.add_argument("--max-new-tokens", type=int, default=128)
    ap.add_argument("--notes", type=int, default=1000)
    a = ap.parse_args()
    from transformers import BertConfig as HFBertConfig, BertModel, LlamaConfig as HFLlamaConfig, LlamaForCausalLM

    from docqa_amd.pipeline.corpus import build_corpus
    from docqa_amd.pipeline.rag import DEFAULT_TEMPLATE
    from docqa_amd.text.synthetic import synthetic_questions
    from docqa_amd.text.tokenizer import ChatTokenizer, WordPieceTokenizer

    dev = "cuda"
    torch.manual_seed(0)
    enc = BertModel(HFBertConfig(vocab_size=30522, hidden_size=384, num_hidden_layers=6, num_attention_heads=12,
                                 intermediate_size=1536)).to(dev).eval()
    cfg = HFLlamaConfig(vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                        num_attention_heads=32, num_key_value_heads=8, rope_theta=500000.0,
                        max_position_embeddings=8192, torch_dtype=torch.bfloat16)
    with torch.device("meta"):
        llm = LlamaForCausalLM(cfg)
    llm = llm.to_empty(device=dev).to(torch.bfloat16)
    with torch.no_grad():
        for p in llm.parameters():
            p.normal_(0.0, 0.02)
    llm.eval()
    wp, chat = WordPieceTokenizer(), ChatTokenizer()
    recs = build_corpus(a.notes)

    @torch.no_grad()
    def embed(texts):
        out = []
        for t in texts:  # sentence-transformers encodes the reference's chunks one by one
            ids = torch.tensor([wp.encode(t)], device=dev)
            h = enc(input_ids=ids).last_hidden_state
            out.append(torch.nn.functional.normalize(h.mean(1), dim=-1))
        return torch.cat(out)

    xb = torch.cat([embed([r["text_content"] for r in recs[i:i + 256]]) for i in range(0, len(recs), 256)])
    qs = synthetic_questions(a.queries + 1, seed=123)
    lat = []
    for i, q in enumerate(qs):
        torch.cuda.synchronize()
        t = time.perf_counter()
        with torch.no_grad():
            e = embed([q])
            d = (xb - e).pow(2).sum(1)
            top = torch.topk(d, 3, largest=False).indices.tolist()
            ctx = "\n\n".join(recs[j]["text_content"] for j in top)
            ids = torch.tensor([chat.chat_prompt(DEFAULT_TEMPLATE.format(context=ctx, question=q))], device=dev)
            out = llm.generate(ids, max_new_tokens=a.max_new_tokens, min_new_tokens=a.max_new_tokens,
                               do_sample=False, use_cache=True, pad_token_id=0)
        torch.cuda.synchronize()
        if i > 0:  # first query = warmup
            lat.append(time.perf_counter() - t)
    print(json.dumps({"metric": "reference_equiv_qa_queries_per_sec", "value": round(len(lat) / sum(lat), 4),
                      "p50_latency_ms": round(1e3 * statistics.median(lat), 1), "queries": len(lat),
                      "max_new_tokens": a.max_new_tokens,
                      "stack": "HF transformers Llama-3-8B generate (bf16, batch 1, SDPA, KV cache) + "
                               "eager MiniLM + torch exact L2 k=3, serial requests"}), flush=True)


if __name__ == "__main__":
    main()
