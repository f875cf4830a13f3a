"""The paged KV pool must not inherit NaN bit patterns from memory an earlier tensor of the
process left behind: the decode kernels stream whole 32-token tiles and zero the masked
positions' probabilities, and 0 x NaN = NaN in P.V (found as an order-dependent failure of
the pipelined-vs-sequential test after the IVF-PQ tests).  The pool is zero-initialised;
here the caching allocator is first filled with NaN garbage and freed, then an engine is
built on that memory and must generate what an engine on clean memory generates."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_engine_on_nan_garbage_memory_matches_clean():
    from docqa_amd import ops
    from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
    from docqa_amd.models.llama import LlamaConfig, LlamaModel

    assert ops.load_native()
    m = LlamaModel(LlamaConfig.preset("llama3-1b-test"), device="cuda", seed=5)
    g = torch.Generator().manual_seed(2)
    prompts = [torch.randint(3, 30000, (n,), generator=g).tolist() for n in (5, 33, 70, 100, 129, 200)]
    params = SamplingParams(max_new_tokens=10, stop_on_eos=False)
    clean = LLMEngine(m, max_batch=8, max_context=512, use_graphs=True)
    ref = clean.generate(prompts, params)
    nkv = sum(k.numel() + v.numel() for k, v in clean.kv.caches)
    del clean
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    # poison: bf16 NaN (0x7fff) over more memory than the pool needs, then hand it back
    junk = torch.full((2 * nkv,), 0x7FFF, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    del junk
    eng = LLMEngine(m, max_batch=8, max_context=512, use_graphs=True)
    assert all(bool(torch.isfinite(k.float()).all()) for k, _ in eng.kv.caches)
    assert eng.generate(prompts, params) == ref
