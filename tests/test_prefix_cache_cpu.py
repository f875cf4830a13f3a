"""Prompt-prefix KV caching (native C++ block manager + paged prefill attention): a
second request sharing a prompt prefix reuses the cached KV blocks and produces exactly
the tokens of an engine without the cache."""
import torch

from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
from docqa_amd.models.llama import LlamaConfig, LlamaModel


def test_prefix_cache_reuse_is_exact():
    m = LlamaModel(LlamaConfig.preset("tiny"), device="cpu", dtype=torch.float32, seed=3)
    eng = LLMEngine(m, max_batch=4, max_context=512, block_size=16, use_graphs=False)
    assert hasattr(eng.kv.allocator, "match_alloc_batch"), "native block manager not loaded"
    pre = list(range(100, 180))                    # 5 full shared blocks
    ps = [pre + [1, 2, 3], pre + [9, 8, 7, 6, 5], pre[:32]]  # last: prompt == 2 full blocks
    sp = SamplingParams(max_new_tokens=5, stop_on_eos=False)
    first = eng.generate(ps, sp)
    assert eng.stats.cached_tokens == 0
    second = eng.generate(ps, sp)
    # whole blocks (80, 80, 16: the last prompt's second block is recomputed) + the
    # token-granular rows of the partial block: every token but the last one is cached
    assert eng.stats.cached_tokens == sum(len(p) - 1 for p in ps)
    assert eng.tail.hit_tokens == 2 + 4 + 15
    ref = LLMEngine(m, max_batch=4, max_context=512, block_size=16, use_graphs=False,
                    prefix_cache=False).generate(ps, sp)
    assert first == second == ref
    eng.tail.clear()   # blocks pinned by the token-granular prefix cache
    st = eng.kv.allocator.stats()
    assert st["free"] + st["evictable"] == eng.kv.num_blocks


def test_prefix_cache_eviction_under_pressure():
    m = LlamaModel(LlamaConfig.preset("tiny"), device="cpu", dtype=torch.float32, seed=4)
    eng = LLMEngine(m, max_batch=2, max_context=128, block_size=16, num_blocks=12, use_graphs=False)
    sp = SamplingParams(max_new_tokens=4, stop_on_eos=False)
    for s in range(6):  # distinct prompts fill the cache; eviction must make room
        p = [s * 7 + i for i in range(60)]
        assert len(eng.generate([p], sp)[0]) == 4


def test_cascade_decode_matches_plain_decode():
    """Cascade decode (shared prompt prefix attended once for the batch, suffixes per row)
    generates exactly the tokens of plain paged decode: a batch whose prompts share 5
    cached blocks switches to the cascade path on its second run."""
    cfg = LlamaConfig(name="tiny-gqa4", vocab_size=4096, hidden=256, intermediate=512, layers=2,
                      heads=8, kv_heads=2, head_dim=128, max_position=2048, bos_token_id=1, eos_token_id=2)
    m = LlamaModel(cfg, device="cpu", dtype=torch.float32, seed=5)
    eng = LLMEngine(m, max_batch=8, max_context=512, block_size=16, use_graphs=False)
    eng.cascade_min_tokens = 32
    pre = list(range(200, 280))                    # 5 full shared blocks
    ps = [pre + [11 + i, 7, 3 * i + 1][: 1 + i % 3] + list(range(i)) for i in range(6)]
    sp = SamplingParams(max_new_tokens=20, stop_on_eos=False)   # crosses block boundaries
    first = eng.generate(ps, sp)
    assert not any(k[2] for k in eng._graphs)
    second = eng.generate(ps, sp)
    assert any(k[2] for k in eng._graphs), "second run must take the cascade path"
    ref = LLMEngine(m, max_batch=8, max_context=512, block_size=16, use_graphs=False,
                    prefix_cache=False).generate(ps, sp)
    assert first == second == ref


def test_cascade_reference_op_equals_paged_decode():
    from docqa_amd.ops import reference as R

    torch.manual_seed(0)
    NB, Hkv, BS, D, Hq, B = 40, 2, 16, 128, 8, 5
    kc, vc = torch.randn(NB, Hkv, BS, D), torch.randn(NB, Hkv, BS, D)
    shared = [3, 7, 1]
    bt = torch.zeros(B, 8, dtype=torch.int32)
    for b in range(B):
        bt[b, :3] = torch.tensor(shared)
        bt[b, 3:] = torch.arange(10 + 5 * b, 15 + 5 * b)
    cl = torch.tensor([49, 60, 80, 100, 120], dtype=torch.int32)
    q = torch.randn(B, (Hq + 2 * Hkv) * D)
    a = R.paged_decode(q, kc, vc, bt, cl, Hq, 128, 0.1)
    c = R.paged_decode_cascade(q, kc, vc, bt, cl, Hq, 128, 0.1, torch.tensor(shared + [0] * 5, dtype=torch.int32),
                               torch.tensor([48], dtype=torch.int32))
    assert torch.allclose(a, c, atol=1e-5)


def test_tail_cache_lookup_register_evict_accounting():
    """TailCache (token-granular prefix reuse): the best variant is found by bisection,
    entries pin their blocks, LRU eviction and shrink return them, and concurrent
    register/lookup from two threads keeps the allocator's accounting exact."""
    import random
    import threading

    from docqa_amd import ops
    from docqa_amd.engine.kv_cache import TailCache, make_allocator

    assert ops.load_native()
    a = make_allocator(256, 16)
    tc = TailCache(a, 16, capacity=40)
    base = list(range(100, 116))                              # one full block
    p1 = base + [1, 2, 3, 4, 5]
    p2 = base + [1, 2, 9, 9]
    t1, t2 = a.alloc(2), a.alloc(2)
    tc.register(p1, t1)
    tc.register(p2, t2)
    # block 1 variants: (1,2,3,4,5) and (1,2,9,9); a prompt continuing 1,2,3,4 matches p1's
    hit = tc.lookup(base + [1, 2, 3, 4, 7, 7], 1, limit=10)
    assert hit == (t1[1], 4)
    tc.unpin([hit[0]])
    assert tc.lookup(base + [5, 5], 1, limit=10) is None       # no variant starts with 5
    hit = tc.lookup(base + [1, 2, 3], 1, limit=2)             # capped by the limit
    assert hit is not None and hit[1] == 2
    tc.unpin([hit[0]])
    a.free(t1)
    a.free(t2)
    tc.clear()
    assert a.num_free() == 256

    errors = []

    def worker(seed):
        r = random.Random(seed)
        try:
            for _ in range(300):
                p = base + [r.randrange(4) for _ in range(r.randrange(1, 30))]
                tb = a.alloc((len(p) + 15) // 16)
                h = tc.lookup(p, 1, len(p) - 17) if len(p) > 17 else None
                if h is not None:
                    tc.unpin([h[0]])
                tc.register(p, tb)
                a.free(tb)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=worker, args=(s,)) for s in (1, 2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors
    assert len(tc) <= 40
    tc.clear()
    assert a.num_free() == 256
