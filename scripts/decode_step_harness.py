"""A batch-256 Llama-3-8B decode on the engine alone (graph-captured steps, no RAG pipeline
threads or side streams): the in-step arm of scripts/instep_vs_isolated_pmc.sh.
python scripts/decode_step_harness.py [new_tokens] [graphs 0|1]"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from docqa_amd import ops  # noqa: E402
from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams  # noqa: E402
from docqa_amd.models.llama import LlamaConfig, LlamaModel  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    graphs = (sys.argv[2] != "0") if len(sys.argv) > 2 else True
    assert ops.load_native()
    m = LlamaModel(LlamaConfig.preset("llama3-8b"), device="cuda")
    eng = LLMEngine(m, max_batch=256, max_context=1024, use_graphs=graphs, kv_mem_fraction=0.5)
    g = torch.Generator().manual_seed(0)
    prompts = [torch.randint(3, 120000, (600,), generator=g).tolist() for _ in range(256)]
    sp = SamplingParams(max_new_tokens=n, stop_on_eos=False)
    eng.generate(prompts, sp)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
