"""Generation engine on CPU (reference ops, fp32 tiny Llama): paged KV cache + varlen
prefill + decode loop must reproduce a naive full-recompute greedy decode, and be
invariant to batching."""
import torch

from docqa_amd.engine.kv_cache import KVCache, PyBlockAllocator
from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
from docqa_amd.models.llama import AttnMeta, LlamaConfig, LlamaModel


def _model():
    return LlamaModel(LlamaConfig.preset("tiny"), device="cpu", dtype=torch.float32, seed=7)


def _naive_greedy(m, prompt, n):
    toks = list(prompt)
    out = []
    for _ in range(n):
        kv = KVCache(m.cfg.layers, 64, m.hkv, m.cfg.head_dim, 16, "cpu", torch.float32)
        T = len(toks)
        meta = AttnMeta(prefill=True, positions=torch.arange(T, dtype=torch.int32),
                        slot_mapping=torch.arange(T, dtype=torch.int32),
                        cu_seqlens=torch.tensor([0, T], dtype=torch.int32), max_len=T)
        logits = m.forward(torch.tensor(toks, dtype=torch.int32), meta, kv.caches,
                           torch.tensor([T - 1]))
        nxt = int(logits[0].argmax())
        out.append(nxt)
        toks.append(nxt)
    return out


def test_engine_matches_naive_recompute():
    m = _model()
    prompts = [[1, 5, 9, 22, 7], [3] * 20 + [4, 5]]
    eng = LLMEngine(m, max_batch=4, max_context=128, block_size=16, use_graphs=False)
    out = eng.generate(prompts, SamplingParams(max_new_tokens=6, stop_on_eos=False))
    for p, o in zip(prompts, out):
        assert o == _naive_greedy(m, p, 6)


def test_engine_batch_invariance_and_block_reuse():
    m = _model()
    prompts = [[2, 3, 4], list(range(10, 60)), [7, 7, 7, 7, 1]]
    eng = LLMEngine(m, max_batch=8, max_context=128, block_size=16, use_graphs=False)
    sp = SamplingParams(max_new_tokens=5, stop_on_eos=False)
    free0 = eng.kv.allocator.num_free()
    batch = eng.generate(prompts, sp)
    single = [eng.generate([p], sp)[0] for p in prompts]
    assert batch == single
    assert eng.kv.allocator.num_free() == free0  # every block returned


def test_engine_max_batch_chunking_and_eos_stop():
    m = _model()
    eng = LLMEngine(m, max_batch=2, max_context=64, block_size=16, use_graphs=False)
    prompts = [[1, 2, 3]] * 5
    out = eng.generate(prompts, SamplingParams(max_new_tokens=3, stop_on_eos=False))
    assert len(out) == 5 and all(o == out[0] for o in out)


def test_context_overflow_rejected():
    m = _model()
    eng = LLMEngine(m, max_batch=2, max_context=32, block_size=16, use_graphs=False)
    try:
        eng.generate([[1] * 30], SamplingParams(max_new_tokens=8))
    except ValueError:
        return
    raise AssertionError("expected ValueError")


def test_py_block_allocator():
    a = PyBlockAllocator(4)
    x = a.alloc(3)
    assert a.num_free() == 1
    a.share(x[:1])
    a.free(x)
    assert a.num_free() == 3
    a.free(x[:1])
    assert a.num_free() == 4
    try:
        a.alloc(5)
    except MemoryError:
        pass
    else:
        raise AssertionError


def test_sampling_reference_topk1_is_greedy():
    from docqa_amd.ops import reference as R

    x = torch.randn(4, 50)
    out = R.sample(x, torch.ones(4), torch.ones(4, dtype=torch.int32), torch.ones(4), torch.rand(4))
    assert torch.equal(out, x.argmax(-1))
