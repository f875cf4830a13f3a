"""Generation engine on CPU (reference ops, fp32 tiny Llama): paged KV cache + varlen
prefill + decode loop must reproduce a naive full-recompute greedy decode, and be
invariant to batching."""
import pytest
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
    if eng.tail is not None:
        eng.tail.clear()   # blocks pinned by the token-granular prefix cache
    assert eng.kv.allocator.num_free() == free0  # every block returned


def test_token_granular_prefix_reuse_identical_tokens():
    """Prompts diverging INSIDE a KV block (RAG chunk / question boundaries): the
    token-granular prefix cache copies the common rows of the block instead of
    recomputing them; greedy tokens equal the no-cache engine's, blocks are accounted."""
    import os

    m = _model()
    base = list(range(10, 47))                       # 2 full 16-token blocks + 5 tokens
    prompts1 = [base + [5, 6, 7, 8], base + [9, 9]]
    prompts2 = [base + [5, 6, 7, 1, 2, 3], base + [9, 4], base[:20] + [3, 3, 3]]
    sp = SamplingParams(max_new_tokens=6, stop_on_eos=False)
    eng = LLMEngine(m, max_batch=8, max_context=128, block_size=16, use_graphs=False)
    if eng.tail is None:
        pytest.skip("prefix cache needs the native block manager")
    free0 = eng.kv.allocator.num_free()
    eng.generate(prompts1, sp)
    c0 = eng.stats.cached_tokens
    got = eng.generate(prompts2, sp)
    # base[32:37] + [5, 6, 7] of prompt 0, base[32:37] + [9] of prompt 1, base[16:20] of prompt 2
    assert eng.stats.cached_tokens - c0 == (32 + 8) + (32 + 6) + (16 + 4)
    assert eng.tail.hit_tokens == 8 + 6 + 4
    os.environ["DOCQA_PREFIX_CACHE"] = "0"
    try:
        ref = LLMEngine(m, max_batch=8, max_context=128, block_size=16, use_graphs=False)
    finally:
        del os.environ["DOCQA_PREFIX_CACHE"]
    assert ref.tail is None
    assert got == ref.generate(prompts2, sp)
    eng.tail.clear()
    assert eng.kv.allocator.num_free() == free0


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


def test_splitk_reference_ops_cpu():
    """CPU references of the fused split-K decode path: partial slabs sum to x @ w^T and
    the consumers see bf16(sum) exactly like the unfused projection."""
    import torch

    from docqa_amd import ops
    from docqa_amd.ops import reference as R

    torch.manual_seed(0)
    x = torch.randn(5, 1024).bfloat16()
    w = torch.randn(256, 1024).bfloat16()
    P = ops.dgemm_partial(x, w, 4)
    assert P.shape == (4, 5, 256)
    assert torch.allclose(P.sum(0), x.float() @ w.float().T, atol=1e-3, rtol=1e-4)
    assert ops.decode_splits(64, 6144, 4096) == 2 and ops.decode_splits(64, 4096, 14336) == 4
    assert ops.decode_splits(64, 28672, 4096) == 0 and ops.decode_splits(64, 128256, 4096) == 0
    # 65-128 rows: 128-row tiles where a split reaches 192 workgroups, else 64-row tiles
    assert ops.decode_plan(128, 6144, 4096) == (4, 128) and ops.decode_plan(128, 4096, 4096) == (4, 64)
    assert ops.decode_plan(128, 4096, 14336) == (4, 64) and ops.decode_plan(100, 28672, 4096)[0] == 0
    assert ops.decode_plan(129, 6144, 4096)[0] == 0
    # 129-192 rows: O / down on 64-row tiles x 4 slabs, QKV / gate|up / LM head on hipBLASLt
    assert ops.decode_plan(192, 4096, 4096) == (4, 64) and ops.decode_plan(160, 4096, 14336) == (4, 64)
    assert ops.decode_plan(192, 28672, 4096)[0] == 0 and ops.decode_plan(193, 4096, 4096)[0] == 0
    r1 = torch.randn(5, 256).bfloat16()
    r2 = r1.clone()
    g = torch.ones(256).bfloat16()
    o1 = ops.add_rmsnorm_splitk(P, r1, g, 1e-5)
    o2 = R.add_rmsnorm(P.sum(0).bfloat16(), r2, g, 1e-5)
    assert torch.equal(r1, r2) and torch.equal(o1, o2)


def test_glu_interleave_roundtrip_cpu():
    import torch

    from docqa_amd.ops import reference as R

    g, u = torch.randn(32, 24), torch.randn(32, 24)
    il = R.glu_interleave(g, u)
    assert torch.equal(il[:8], g[:8]) and torch.equal(il[8:16], u[:8]) and torch.equal(il[16:24], g[8:16])
    g2, u2 = R.glu_split(il)
    assert torch.equal(g, g2) and torch.equal(u, u2)
    x = torch.randn(3, 24)
    a = R.silu_mul(torch.cat([x @ g.T, x @ u.T], -1))
    b = R.silu_mul(x @ il.T, interleaved=True)
    assert torch.allclose(a, b, atol=1e-5)


def test_chunked_prefill_matches_single_pass():
    """A prompt longer than max_prefill_tokens is prefilled in pieces through the paged
    prefix attention; the greedy continuation must equal the one-pass prefill's."""
    m = _model()
    prompts = [list(range(3, 103)), [5, 6, 7], list(range(200, 150, -1))]
    sp = SamplingParams(max_new_tokens=6, stop_on_eos=False)
    one = LLMEngine(m, max_batch=4, max_context=256, block_size=16, use_graphs=False,
                    prefix_cache=False).generate(prompts, sp)
    chunked = LLMEngine(m, max_batch=4, max_context=256, block_size=16, use_graphs=False,
                        max_prefill_tokens=32, prefix_cache=False).generate(prompts, sp)
    assert one == chunked
    assert one[0] == _naive_greedy(m, prompts[0], 6)


def test_lpt_dispatch_order_and_decode_state_ops():
    """set_order: active rows longest-context first, then the padded rows (a permutation of
    the bucket); re-uploaded only when the batch key changes.  decode_slots /
    decode_advance references: slot = block * BS + offset (-1 for padded rows)."""
    from docqa_amd import ops
    from docqa_amd.engine.llm_engine import _DecodeGraph

    m = LlamaModel(LlamaConfig.preset("tiny"), device="cpu")
    eng = LLMEngine(m, max_batch=8, max_context=128, block_size=16, use_graphs=False)
    g = _DecodeGraph(eng, 8)
    eng.set_order(g, [30, 90, 10, 50, 70], key=1)
    assert g.order.tolist() == [1, 4, 3, 0, 2, 5, 6, 7]
    g.order.fill_(0)
    eng.set_order(g, [1, 2, 3], key=1)          # same key: untouched
    assert g.order.tolist() == [0] * 8
    eng.set_order(g, [1, 2, 3], key=2)
    assert g.order.tolist() == [2, 1, 0, 3, 4, 5, 6, 7]

    bt = torch.tensor([[5, 6, 7], [8, 9, 10]], dtype=torch.int32)
    pos = torch.tensor([17, 3], dtype=torch.int32)
    valid = torch.tensor([1, 0], dtype=torch.int32)
    assert ops.decode_slots(bt, pos, valid, 16).tolist() == [6 * 16 + 1, -1]
    out, tok = torch.zeros(2, dtype=torch.long), torch.zeros(2, dtype=torch.int32)
    ctx = pos + 1
    ops.decode_advance(torch.tensor([11, 12]), out, tok, pos, ctx, valid)
    assert out.tolist() == [11, 12] and tok.tolist() == [11, 12]
    assert pos.tolist() == [18, 3] and ctx.tolist() == [19, 4]


def test_token_cls_argmax_reference_cpu():
    """CPU path of the fused NER head + argmax: padded label rows never win."""
    import torch

    from docqa_amd import ops

    h = torch.randn(33, 64)
    w = torch.zeros(16, 64)
    w[:9] = torch.randn(9, 64)
    b = torch.zeros(16)
    b[9:] = 1e9  # would win if the padded rows were not excluded
    got = ops.token_cls_argmax(h, w, b, 9)
    assert torch.equal(got, (h @ w[:9].t() + b[:9]).argmax(-1))


def test_pack_decode_groups_covers_rows_and_keeps_clusters():
    """Every row in exactly one group of <= 4; rows sharing their first block past the
    cascade prefix share a group when the cluster fits; LPT order (most blocks first)."""
    from docqa_amd import ops

    skip = 2
    tables = [[0, 1, 10, 11, 50], [0, 1, 10, 11, 51], [0, 1, 20, 52, 53], [0, 1, 10, 12, 54],
              [0, 1, 30, 55, 56], [0, 1, 20, 57, 58], [0, 1, 60, 61, 62]]
    lens = [300] * len(tables)
    quads = ops.pack_decode_groups(tables, lens, skip, 64, cap=4)
    assert sorted(r for q in quads for r in q) == list(range(len(tables)))
    assert all(1 <= len(q) <= 4 for q in quads)
    where = {r: i for i, q in enumerate(quads) for r in q}
    assert where[0] == where[1] == where[3]          # cluster of first block 10
    assert where[2] == where[5]                      # cluster of first block 20
    work = [len({b for r in q for b in tables[r][skip:5]}) for q in quads]
    assert work == sorted(work, reverse=True)
    # too many groups for the cap: consecutive quads of the sorted rows
    quads = ops.pack_decode_groups(tables, lens, skip, 64, cap=1)
    assert sorted(r for q in quads for r in q) == list(range(len(tables)))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_pack_decode_groups_ignores_physical_block_ids(seed):
    """The packing (and so the split plan and every row's partial-merge order) depends only
    on which rows share blocks: renaming the physical blocks -- as a pipelined run's
    timing-dependent free / reserve order does -- yields the same groups and plan."""
    import random

    from docqa_amd import ops

    skip = 2
    tables = [[0, 1, 10, 11, 50, 70], [0, 1, 10, 11, 51, 71], [0, 1, 20, 52, 53, 72], [0, 1, 10, 12, 54, 73],
              [0, 1, 30, 55, 56, 74], [0, 1, 20, 57, 58, 75], [0, 1, 60, 61, 62, 76], [0, 1, 30, 77, 78, 79]]
    lens = [330, 300, 370, 250, 384, 200, 310, 290]
    ids = sorted({b for t in tables for b in t})
    perm = dict(zip(ids, random.Random(seed).sample(range(1000, 2000), len(ids))))
    renamed = [[perm[b] for b in t] for t in tables]
    for cap in (2, 4):
        q1 = ops.pack_decode_groups(tables, lens, skip, 64, cap)
        q2 = ops.pack_decode_groups(renamed, lens, skip, 64, cap)
        assert q1 == q2
        p1 = ops.split_decode_groups(q1, tables, lens, skip, 64, cap=16, tiles_per_item=3)
        p2 = ops.split_decode_groups(q2, renamed, lens, skip, 64, cap=16, tiles_per_item=3)
        assert torch.equal(p1, p2)


@pytest.mark.parametrize("tiles", [1, 2, 5, 100])
def test_split_decode_groups_plan(tiles):
    """Split plan: each group's block positions past the prefix are covered by its items
    exactly once (contiguous ranges), split groups own consecutive partial slots listed in
    a merge row, unsplit groups finish in place (slot -1), items are largest first, and
    the tile budget is respected wherever a cut was possible."""
    from docqa_amd import ops

    skip = 2
    tables = [[0, 1, 10, 11, 50, 70], [0, 1, 10, 11, 51, 71], [0, 1, 20, 52, 53, 72], [0, 1, 10, 12, 54, 73],
              [0, 1, 30, 55, 56, 74], [0, 1, 20, 57, 58, 75], [0, 1, 60, 61, 62, 76]]
    lens = [330, 300, 370, 250, 384, 200, 310]
    quads = ops.pack_decode_groups(tables, lens, skip, 64, cap=4)
    plan = ops.split_decode_groups(quads, tables, lens, skip, 64, cap=16, tiles_per_item=tiles)
    assert plan.shape == (2, 16, 8) and plan.dtype == torch.int32
    items = [r.tolist() for r in plan[0] if (r[:4] >= 0).any()]
    merges = [r.tolist() for r in plan[1] if r[5] > 0]
    slots = sorted(it[6] for it in items if it[6] >= 0)
    assert slots == list(range(len(slots)))
    for qd in quads:
        key = sorted(qd)
        mine = [it for it in items if sorted(r for r in it[:4] if r >= 0) == key]
        nb = max((lens[r] + 63) // 64 for r in qd)
        cover = []
        for it in sorted(mine, key=lambda it: it[4]):
            cover += list(range(max(it[4], skip), min(it[5], nb)))
        assert cover == list(range(skip, nb))
        if len(mine) == 1:
            assert mine[0][6] == -1
        else:
            mg = [m for m in merges if sorted(r for r in m[:4] if r >= 0) == key]
            assert len(mg) == 1 and mg[0][5] == len(mine)
            assert sorted(it[6] for it in mine) == list(range(mg[0][4], mg[0][4] + len(mine)))
            per = dict(ops.group_tiles_by_position(tables, lens, qd, skip, 64))
            for it in mine:
                t = sum(per.get(p, 0) for p in range(it[4], min(it[5], nb)))
                single = it[5] - it[4] == 1
                assert t <= tiles or single
    if tiles == 1:
        assert merges
    if tiles == 100:
        assert not merges


@pytest.mark.parametrize("tiles", [1, 2, 100])
def test_deferred_split_plan(tiles):
    """Deferred split plan (prefix kernel forked beside the group kernel): the same items
    as the plain split plan, but every item writes a partial and every group -- split or
    not -- has one merge row over its consecutive slots, so nothing reads the prefix
    partials before the merge."""
    from docqa_amd import ops

    skip = 2
    tables = [[0, 1, 10, 11, 50, 70], [0, 1, 10, 11, 51, 71], [0, 1, 20, 52, 53, 72], [0, 1, 10, 12, 54, 73],
              [0, 1, 30, 55, 56, 74], [0, 1, 20, 57, 58, 75], [0, 1, 60, 61, 62, 76]]
    lens = [330, 300, 370, 250, 384, 200, 310]
    quads = ops.pack_decode_groups(tables, lens, skip, 64, cap=4)
    plain = ops.split_decode_groups(quads, tables, lens, skip, 64, cap=16, tiles_per_item=tiles)
    plan = ops.split_decode_groups(quads, tables, lens, skip, 64, cap=16, tiles_per_item=tiles, defer=True)
    assert plan.shape == (2, 16, 8)
    items = [r.tolist() for r in plan[0] if (r[:4] >= 0).any()]
    # the same work items (rows; an unsplit group's range is explicit instead of open-ended)
    assert sorted(it[:4] for it in items) == sorted(r[:4].tolist() for r in plain[0] if (r[:4] >= 0).any())
    assert sorted(it[6] for it in items) == list(range(len(items)))
    merges = [r.tolist() for r in plan[1] if r[5] > 0]
    assert len(merges) == len(quads)
    for m in merges:
        key = sorted(r for r in m[:4] if r >= 0)
        mine = [it for it in items if sorted(r for r in it[:4] if r >= 0) == key]
        assert sorted(it[6] for it in mine) == list(range(m[4], m[4] + m[5]))


@pytest.mark.parametrize("tiles,bins", [(1, 3), (2, 4), (5, 2), (100, 8)])
def test_persistent_decode_plan(tiles, bins):
    """Persistent plan [3, cap, 8]: every item owns slot = its index, every group has one
    merge row over its consecutive slots, items tile each group's positions exactly once,
    and the bins hold every item once with <= 8 items / <= 512 tiles, LPT-balanced."""
    from docqa_amd import ops

    skip = 2
    tables = [[0, 1, 10, 11, 50, 70], [0, 1, 10, 11, 51, 71], [0, 1, 20, 52, 53, 72], [0, 1, 10, 12, 54, 73],
              [0, 1, 30, 55, 56, 74], [0, 1, 20, 57, 58, 75], [0, 1, 60, 61, 62, 76]]
    lens = [330, 300, 370, 250, 384, 200, 310]
    quads = ops.pack_decode_groups(tables, lens, skip, 64, cap=4)
    plan = ops.split_decode_groups(quads, tables, lens, skip, 64, cap=16, tiles_per_item=tiles, bins=bins)
    assert plan.shape == (3, 16, 8)
    items = [r.tolist() for r in plan[0] if r[6] >= 0]
    assert [it[6] for it in items] == list(range(len(items)))
    merges = [r.tolist() for r in plan[1] if r[5] > 0]
    assert len(merges) == len(quads)
    for qd in quads:
        key = sorted(qd)
        mg = [m for m in merges if sorted(r for r in m[:4] if r >= 0) == key]
        assert len(mg) == 1
        mine = items[mg[0][4]:mg[0][4] + mg[0][5]]
        assert all(sorted(r for r in it[:4] if r >= 0) == key for it in mine)
        nb = max((lens[r] + 63) // 64 for r in qd)
        cover = []
        for it in mine:
            cover += list(range(max(it[4], skip), min(it[5], nb)))
        assert cover == list(range(skip, nb))
    binned = [int(i) for i in plan[2].flatten() if i >= 0]
    assert sorted(binned) == list(range(len(items)))
    assert all(int((plan[2, b] >= 0).sum()) <= ops.BIN_ITEMS for b in range(16))
    assert int((plan[2, :, 0] >= 0).sum()) == min(bins, len(items))
    assert ops.persist_bins(256, 8) == 96 and ops.persist_bins(512, 8) == 128 and ops.persist_bins(4, 2) == 4


def test_persistent_identity_plan_cpu(monkeypatch):
    from docqa_amd import ops
    from docqa_amd.engine.llm_engine import _identity_groups

    monkeypatch.setenv("DOCQA_GROUP_PERSIST", "1")
    g = _identity_groups(256, "cpu", 8)
    assert g.shape == (3, 256, 8)
    items = g[0][g[0, :, 6] >= 0]
    assert items.shape[0] == 64 and items[:, :4].flatten().tolist() == list(range(256))
    assert (g[1, :64, 5] == 1).all() and (g[1, :64, 4] == torch.arange(64)).all()
    assert sorted(int(i) for i in g[2].flatten() if i >= 0) == list(range(64))
    assert int((g[2, :, 1] >= 0).sum()) == 0          # one quad per bin
    assert ops.persist_bins(256, 8) >= 64


@pytest.mark.parametrize("defer", [False, True])
def test_split_identity_plan_cpu(monkeypatch, defer):
    """Default (split) identity plan: consecutive quads; deferred: each quad writes slot i
    and has merge row i (nothing reads the forked prefix kernel's partials)."""
    from docqa_amd.engine.llm_engine import _identity_groups

    monkeypatch.setenv("DOCQA_GROUP_PERSIST", "0")
    monkeypatch.setenv("DOCQA_GROUP_DEFER", "1" if defer else "0")
    g = _identity_groups(256, "cpu", 8)
    assert g.shape == (2, 256, 8)
    assert g[0, :64, :4].flatten().tolist() == list(range(256))
    if defer:
        assert (g[0, :64, 6] == torch.arange(64)).all()
        assert (g[1, :64, 5] == 1).all() and (g[1, :64, 4] == torch.arange(64)).all()
    else:
        assert (g[0, :, 6] == -1).all() and (g[1, :, 5] == 0).all()


def test_mid_plan_glu_never_picks_narrow_tiles():
    """the fused-SwiGLU gate|up launch has no 64-wide (cfg 7) variant."""
    from docqa_amd import ops

    for M, N, K in [(256, 1024, 256), (256, 28672, 4096), (512, 2048, 1024), (384, 4096, 512)]:
        S, cfg = ops.mid_plan(M, N, K, glu=True)
        assert cfg != 7
        S2, cfg2 = ops.mid_plan(M, N, K)
        assert S2 >= 1 or cfg2 == 0


def test_prefill_plans_are_hand_written():
    """No library GEMM on the prefill path (VERDICT r5 missing #1): the mid-M shapes the
    round-5 hipBLASLt routes covered take split-K slabs into their consumers, the mid-M
    kernel on the two measured exceptions, or the 256 x 256 tiles
    (profiles/r6_prefill_mid_plans.log); prefill_route never names the library."""
    from docqa_amd import ops

    assert not hasattr(ops, "lib_route") and not hasattr(ops, "_LIB_ROUTES")
    sp = ops.prefill_split_plan
    # 70B TP-8 gate|up shard: SwiGLU consumer over 4 / 2 slabs, the fused epilogue beyond
    assert sp(512, 7168, 8192, glu=True) == 4 and sp(768, 7168, 8192, glu=True) == 2
    assert sp(1024, 7168, 8192, glu=True) == 2 and sp(1536, 7168, 8192, glu=True) == 0
    assert sp(256, 7168, 8192, glu=True) == 0                     # decode-sized: mid-M SwiGLU kernel
    # 8B: down S=4 / 2, QKV S=2 to 1024 rows, O S=4 at 768
    assert sp(768, 4096, 14336) == 4 and sp(1536, 4096, 14336) == 2 and sp(2048, 4096, 14336) == 2
    assert sp(768, 6144, 4096) == 2 and sp(1536, 6144, 4096) == 0 and sp(768, 4096, 4096) == 4
    assert sp(512, 6144, 4096) == 0 and sp(256, 4096, 14336) == 0  # <= 512 rows: mid_plan
    assert sp(512, 1280, 8192) == 8 and sp(4096, 1280, 8192) == 2  # narrow TP shard, any M
    assert sp(700, 28672, 4096, glu=True) == 0                     # enough tiles: fused epilogue
    # the measured mid-M exceptions, and the split deferring to prefill_split_plan
    assert ops.prefill_plan(900, 4096, 4096) == (2, 2) and ops.prefill_plan(900, 8192, 3584) == (1, 2)
    assert ops.prefill_plan(600, 8192, 3584) == (0, 0) and sp(600, 8192, 3584) == 2
    assert ops.prefill_plan(1536, 4096, 14336) == (0, 0)
    assert ops.down_small_split(512, 4096, 14336) == 8 and ops.down_small_split(512, 8192, 3584) == 0
    assert ops.down_small_split(256, 4096, 14336) == 0
    for M in (300, 512, 600, 768, 1024, 1200, 1536, 2048, 4096):
        for N, K, glu in [(6144, 4096, False), (4096, 4096, False), (28672, 4096, True), (4096, 14336, False),
                          (1280, 8192, False), (8192, 1024, False), (7168, 8192, True), (8192, 3584, False)]:
            label, _ = ops.prefill_route(M, N, K, glu=glu, down=K in (14336, 3584))
            assert "hipblaslt" not in label and "linear(" not in label, (M, N, K, label)


def test_reserve_rolls_back_without_prefix_cache():
    """a batch that does not fit frees what it had reserved (prefix cache off)."""
    m = _model()
    eng = LLMEngine(m, max_batch=4, max_context=256, use_graphs=False, num_blocks=6, prefix_cache=False)
    free0 = eng.kv.allocator.num_free()
    prompts = [[5] * 100, [6] * 100, [7] * 100, [8] * 100]     # 2 blocks each with 16 new tokens
    with pytest.raises(MemoryError):
        eng.reserve(prompts, SamplingParams(max_new_tokens=16))
    assert eng.kv.allocator.num_free() == free0


def test_grouped_decode_window_follows_the_rows_not_the_table():
    """The grouped decode kernels cover ops.GROUP_MAX_BLOCKS block positions per work item.
    With a block table sized for a long MAX_CONTEXT (the llm-qa service: 8192 tokens) the
    decision follows the rows' own end lengths -- RAG prompts of ~1k tokens keep the grouped
    kernels -- and a graph built for rows that do not fit never gets decode groups."""
    from docqa_amd import ops
    from docqa_amd.engine.llm_engine import LLMEngine

    m = _model()
    short = LLMEngine(m, max_batch=4, max_context=128, block_size=16, use_graphs=False)
    assert short.max_blocks_per_seq <= ops.GROUP_MAX_BLOCKS and short.groups_fit([10 ** 6])
    long_ = LLMEngine(m, max_batch=4, max_context=2048, block_size=16, use_graphs=False)
    assert long_.max_blocks_per_seq > ops.GROUP_MAX_BLOCKS
    assert long_.groups_fit([900, 1024]) and not long_.groups_fit([900, 1025])
    g_fit = long_._get_graph(4, True, True, True)
    g_long = long_._get_graph(4, True, True, False)
    assert g_fit is not g_long and g_fit.groups_fit and not g_long.groups_fit
    assert short._get_graph(4, True, True, False).groups_fit      # a narrow table always fits
    assert not long_.group_without_prefix(64, fit=False)


def test_mgemm_partial_bf16_slabs_cpu():
    """bf16 split-K slabs (ops.SLAB_BF16): each slab is the fp32 slab rounded once, and the
    consumers sum them in fp32."""
    import torch
    from docqa_amd import ops

    g = torch.Generator().manual_seed(0)
    x = torch.randn(8, 256, generator=g).bfloat16()
    w = (torch.randn(64, 256, generator=g) / 16).bfloat16()
    P32 = ops.mgemm_partial(x, w, 4)
    P16 = ops.mgemm_partial(x, w, 4, bf16=True)
    assert P16.dtype == torch.bfloat16 and P16.shape == (4, 8, 64)
    assert torch.equal(P16, P32.bfloat16())
    res = torch.randn(8, 64, generator=g).bfloat16()
    gam = torch.ones(64).bfloat16()
    r1, r2 = res.clone(), res.clone()
    o16 = ops.add_rmsnorm_splitk(P16, r1, gam, 1e-5)
    o32 = ops.add_rmsnorm_splitk(P16.float(), r2, gam, 1e-5)
    assert torch.equal(o16, o32) and torch.equal(r1, r2)
