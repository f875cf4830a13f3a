"""Does a batch's prefill hide under the previous batch's decode?  Times, on one GPU with
Llama-3-8B: generate(A) alone, prefill(B) alone, and generate(A) on the main stream with
prefill(B) concurrently on a side stream from a helper thread (the shape of a pipelined
prefill).  Prompts: shared 320-token head + distinct tail, 128 new tokens."""
import sys
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch

from docqa_amd import ops
from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
from docqa_amd.models.llama import LlamaConfig, LlamaModel


def main():
    B, P, SH, GEN = int(sys.argv[1]) if len(sys.argv) > 1 else 192, 600, 320, 128
    assert ops.load_native()
    cfg = LlamaConfig.preset("llama3-8b")
    m = LlamaModel(cfg, device="cuda")
    eng = LLMEngine(m, max_batch=B, max_context=2048, num_blocks=3 * B * 32 + 1)
    g = torch.Generator().manual_seed(0)
    head = torch.randint(0, cfg.vocab_size, (SH,), generator=g).tolist()

    def batch():
        return [head + torch.randint(0, cfg.vocab_size, (P - SH,), generator=g).tolist() for _ in range(B)]

    sp = SamplingParams(max_new_tokens=GEN, stop_on_eos=False)
    alloc = eng.kv.allocator

    def prefill(prompts, stream):
        tables, cached = [], []
        for p in prompts:
            hit = alloc.match_prefix(p)
            if hit and len(hit) * eng.block_size >= len(p):
                alloc.free([hit[-1]])
                hit = hit[:-1]
            cached.append(len(hit) * eng.block_size)
            tables.append(hit + alloc.alloc(eng.kv.blocks_for(len(p) + GEN) - len(hit)))
        with torch.inference_mode(), torch.cuda.stream(stream):
            eng._prefill(prompts, tables, cached)
        stream.synchronize()
        for tb in tables:
            alloc.free(tb)

    side = torch.cuda.Stream()
    eng.generate(batch(), sp)                       # graphs, tuning
    prefill(batch(), side)
    for it in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        eng.generate(batch(), sp)
        torch.cuda.synchronize()
        t_gen = time.perf_counter() - t
        t = time.perf_counter()
        prefill(batch(), side)
        t_pre = time.perf_counter() - t
        nb = batch()
        th = threading.Thread(target=prefill, args=(nb, side))
        torch.cuda.synchronize()
        t = time.perf_counter()
        th.start()
        eng.generate(batch(), sp)
        torch.cuda.synchronize()
        th.join()
        t_both = time.perf_counter() - t
        print(f"iter {it}: generate {t_gen*1e3:.0f} ms, prefill {t_pre*1e3:.0f} ms, sum {1e3*(t_gen+t_pre):.0f}; "
              f"concurrent {t_both*1e3:.0f} ms -> hidden {1e3*(t_gen+t_pre-t_both):.0f} ms", flush=True)


if __name__ == "__main__":
    main()
