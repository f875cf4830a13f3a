"""Quick generator probe: Llama-3 random-init prefill/decode timing on one GPU."""
import argparse
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch

from docqa_amd import ops
from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
from docqa_amd.models.llama import LlamaConfig, LlamaModel


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--gen", type=int, default=128)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--max-context", type=int, default=0)
    ap.add_argument("--shared", type=int, default=0, help="leading prompt tokens shared by every request (RAG template)")
    a = ap.parse_args()
    assert ops.load_native()
    cfg = LlamaConfig.preset(a.model)
    t = time.time()
    m = LlamaModel(cfg, device="cuda")
    torch.cuda.synchronize()
    print(f"init {time.time()-t:.1f}s weights {m.weight_bytes()/1e9:.1f} GB", flush=True)
    eng = LLMEngine(m, max_batch=a.batch, max_context=a.max_context or (a.prompt + a.gen + 64),
                    use_graphs=not a.no_graph)
    g = torch.Generator().manual_seed(0)
    head = torch.randint(0, cfg.vocab_size, (a.shared,), generator=g).tolist()
    prompts = [head + torch.randint(0, cfg.vocab_size, (a.prompt - a.shared,), generator=g).tolist()
               for _ in range(a.batch)]
    sp = SamplingParams(max_new_tokens=a.gen, stop_on_eos=False)
    for it in range(a.iters + 1):
        eng.stats.__init__()
        torch.cuda.synchronize()
        t = time.time()
        out = eng.generate(prompts, sp)
        torch.cuda.synchronize()
        dt = time.time() - t
        s = eng.stats
        casc = any(k[2] for k in eng._graphs if isinstance(k, tuple))
        print(f"cascade={casc} cached={s.cached_tokens} ", end="")
        print(f"iter {it}: total {dt*1e3:.0f} ms prefill {s.prefill_s*1e3:.0f} ms "
              f"({s.prompt_tokens/s.prefill_s:.0f} tok/s) decode {s.decode_s*1e3:.0f} ms "
              f"({(a.gen-1)} steps, {s.decode_s/(a.gen-1)*1e3:.2f} ms/step) "
              f"QPS {a.batch/dt:.1f}", flush=True)
    print("sample:", out[0][:16])


if __name__ == "__main__":
    main()
