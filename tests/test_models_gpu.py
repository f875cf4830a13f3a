"""Model-level numerics: whole forwards on the native gfx950 kernels vs the same forward
routed through the fp32 PyTorch reference ops (same weights, same GPU).

Random-init decoders have nearly flat logits, so greedy token streams are compared only
where kernels are identical (graph vs eager); across kernel implementations the tests
compare logits (teacher forcing), which is what numerics parity means."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def native():
    from docqa_amd import ops

    assert ops.load_native(build_if_missing=True)
    return ops


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max()).item()


@pytest.mark.parametrize("preset", ["minilm-l6", "bge-base"])
def test_bert_encoder_native_vs_reference(native, preset):
    from docqa_amd.models.bert import BertConfig, BertEncoder

    enc = BertEncoder(BertConfig.preset(preset), device="cuda")
    g = torch.Generator().manual_seed(0)
    toks = [torch.randint(0, 30000, (n,), generator=g).tolist() for n in (5, 64, 200, 17)]
    e1 = enc.encode(toks)
    with native.use_reference():
        e2 = enc.encode(toks)
    cos = torch.nn.functional.cosine_similarity(e1, e2, dim=1)
    assert cos.min().item() > 0.995, cos


def _prefill_logits(m, kv, prompts, BS):
    from docqa_amd.models.llama import AttnMeta

    ids, pos, slots, cu = [], [], [], [0]
    nb = 0
    tables = []
    for p in prompts:
        n = len(p)
        blocks = list(range(nb, nb + (n + BS) // BS + 1))
        nb += len(blocks)
        tables.append(blocks)
        ids += p
        pos += list(range(n))
        slots += [blocks[t // BS] * BS + t % BS for t in range(n)]
        cu.append(cu[-1] + n)
    meta = AttnMeta(prefill=True, positions=torch.tensor(pos, dtype=torch.int32, device="cuda"),
                    slot_mapping=torch.tensor(slots, dtype=torch.int32, device="cuda"),
                    cu_seqlens=torch.tensor(cu, dtype=torch.int32, device="cuda"),
                    max_len=max(len(p) for p in prompts))
    last = torch.tensor(cu[1:], device="cuda") - 1
    logits = m.forward(torch.tensor(ids, dtype=torch.int32, device="cuda"), meta, kv, last)
    return logits, tables


def _decode_logits(m, kv, prompts, tables, next_tok, BS):
    from docqa_amd.models.llama import AttnMeta

    B = len(prompts)
    maxb = max(len(t) for t in tables)
    bt = torch.zeros(B, maxb, dtype=torch.int32)
    for i, t in enumerate(tables):
        bt[i, :len(t)] = torch.tensor(t)
    lens = [len(p) for p in prompts]
    slots = [tables[i][lens[i] // BS] * BS + lens[i] % BS for i in range(B)]
    meta = AttnMeta(prefill=False, positions=torch.tensor(lens, dtype=torch.int32, device="cuda"),
                    slot_mapping=torch.tensor(slots, dtype=torch.int32, device="cuda"),
                    block_tables=bt.cuda(),
                    context_lens=torch.tensor([n + 1 for n in lens], dtype=torch.int32, device="cuda"),
                    max_context=maxb * BS)
    return m.forward(torch.tensor(next_tok, dtype=torch.int32, device="cuda"), meta, kv)


def test_llama_prefill_decode_logits_native_vs_reference(native):
    from docqa_amd.engine.kv_cache import KVCache
    from docqa_amd.models.llama import LlamaConfig, LlamaModel

    m = LlamaModel(LlamaConfig.preset("llama3-1b-test"), device="cuda")
    g = torch.Generator().manual_seed(1)
    prompts = [torch.randint(0, 32000, (n,), generator=g).tolist() for n in (9, 130, 300)]
    BS = 64
    nxt = [5, 6, 7]
    kv1 = KVCache(m.cfg.layers, 64, m.hkv, m.cfg.head_dim, BS).caches
    kv2 = KVCache(m.cfg.layers, 64, m.hkv, m.cfg.head_dim, BS).caches
    p1, tables = _prefill_logits(m, kv1, prompts, BS)
    d1 = _decode_logits(m, kv1, prompts, tables, nxt, BS)
    with native.use_reference():
        p2, _ = _prefill_logits(m, kv2, prompts, BS)
        d2 = _decode_logits(m, kv2, prompts, tables, nxt, BS)
    assert _rel(p1, p2) < 0.03
    assert _rel(d1, d2) < 0.03


@pytest.mark.parametrize("lens", [(300, 200), (700, 300), (900, 800, 100)])
def test_llama_mid_prefill_plans_vs_reference(native, lens):
    """Prefills of 257..2048 tokens on the mid-M split-K plans (ops.prefill_plan and the short
    prefill's decode plans) track the fp32 reference forward."""
    from docqa_amd.engine.kv_cache import KVCache
    from docqa_amd.models.llama import LlamaConfig, LlamaModel

    m = LlamaModel(LlamaConfig.preset("llama3-1b-test"), device="cuda", seed=8)
    g = torch.Generator().manual_seed(9)
    prompts = [torch.randint(0, 32000, (n,), generator=g).tolist() for n in lens]
    BS = 64
    kv1 = KVCache(m.cfg.layers, 64, m.hkv, m.cfg.head_dim, BS).caches
    kv2 = KVCache(m.cfg.layers, 64, m.hkv, m.cfg.head_dim, BS).caches
    p1, tables = _prefill_logits(m, kv1, prompts, BS)
    d1 = _decode_logits(m, kv1, prompts, tables, [3] * len(prompts), BS)
    with native.use_reference():
        p2, _ = _prefill_logits(m, kv2, prompts, BS)
        d2 = _decode_logits(m, kv2, prompts, tables, [3] * len(prompts), BS)
    assert _rel(p1, p2) < 0.03
    assert _rel(d1, d2) < 0.03


def test_llama_prefill_trim_last_layer(native, monkeypatch):
    """Prefill over a cached prefix with logits for each prompt's last token: the last layer
    run on those rows only (attention as decode attention over the paged cache) == the full
    last layer, and the KV cache written identically."""
    from docqa_amd.engine.kv_cache import KVCache
    from docqa_amd.models import llama as LM

    m = LM.LlamaModel(LM.LlamaConfig.preset("llama3-1b-test"), device="cuda", seed=12)
    g = torch.Generator().manual_seed(13)
    BS, P = 64, 128
    shared = torch.randint(0, 32000, (P,), generator=g).tolist()
    suffixes = [torch.randint(0, 32000, (n,), generator=g).tolist() for n in (37, 300, 5, 900)]
    out = {}
    for trim in (True, False):
        monkeypatch.setattr(LM, "_PREFILL_TRIM", trim)
        kv = KVCache(m.cfg.layers, 128, m.hkv, m.cfg.head_dim, BS).caches
        _prefill_logits(m, kv, [shared], BS)                # blocks 0, 1 (+ spare) hold the prefix
        nb, tables, ids, pos, slots, cu = 3, [], [], [], [], [0]
        for sfx in suffixes:
            own = list(range(nb, nb + (len(sfx) + BS - 1) // BS + 1))
            nb += len(own)
            tb = [0, 1] + own
            tables.append(tb)
            for t in range(P, P + len(sfx)):
                pos.append(t)
                slots.append(tb[t // BS] * BS + t % BS)
            ids += sfx
            cu.append(cu[-1] + len(sfx))
        maxb = max(len(t) for t in tables)
        bt = torch.zeros(len(tables), maxb, dtype=torch.int32)
        for r, t in enumerate(tables):
            bt[r, :len(t)] = torch.tensor(t)
        meta = LM.AttnMeta(prefill=True, positions=torch.tensor(pos, dtype=torch.int32, device="cuda"),
                           slot_mapping=torch.tensor(slots, dtype=torch.int32, device="cuda"),
                           cu_seqlens=torch.tensor(cu, dtype=torch.int32, device="cuda"),
                           max_len=max(len(x) for x in suffixes))
        meta.block_tables = bt.cuda()
        meta.prefix_lens = torch.full((len(suffixes),), P, dtype=torch.int32, device="cuda")
        last = torch.tensor(cu[1:], device="cuda") - 1
        logits = m.forward(torch.tensor(ids, dtype=torch.int32, device="cuda"), meta, kv, last)
        out[trim] = (logits.float(), [c.clone() for pair in kv for c in pair])
    assert _rel(out[True][0], out[False][0]) < 0.02
    for a, b in zip(out[True][1], out[False][1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("slab16,glu16", [(False, False), (True, False), (True, True)])
def test_llama_mid_batch_decode_native_vs_reference(native, monkeypatch, slab16, glu16):
    """A 256-row decode step (the mid-M GEMM path: split-K QKV / O / down slabs -- fp32, or
    bf16 with ``slab16`` (ops.SLAB_BF16) -- fused SwiGLU, fused LM-head argmax) against the
    same step on the fp32 reference ops."""
    from docqa_amd.engine.kv_cache import KVCache
    from docqa_amd.models.llama import LlamaConfig, LlamaModel

    monkeypatch.setattr(native, "SLAB_BF16", slab16)
    monkeypatch.setattr(native, "_GLU_SPLIT16", glu16)

    m = LlamaModel(LlamaConfig.preset("llama3-1b-test"), device="cuda", seed=5)
    assert native.mid_plan(256, *m.layers[0]["qkv"].shape)[0] > 0
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, 32000, (int(n),), generator=g).tolist()
               for n in torch.randint(3, 90, (256,), generator=g)]
    BS = 64
    nxt = torch.randint(0, 32000, (256,), generator=g).tolist()
    kv1 = KVCache(m.cfg.layers, 800, m.hkv, m.cfg.head_dim, BS).caches
    kv2 = KVCache(m.cfg.layers, 800, m.hkv, m.cfg.head_dim, BS).caches
    _, tables = _prefill_logits(m, kv1, prompts, BS)
    d1 = _decode_logits(m, kv1, prompts, tables, nxt, BS)
    with native.use_reference():
        _prefill_logits(m, kv2, prompts, BS)
        d2 = _decode_logits(m, kv2, prompts, tables, nxt, BS)
    assert _rel(d1, d2) < 0.03
    # fused LM head + argmax on the same step == argmax of the bf16 logits (up to near-ties)
    _prefill_logits(m, kv1, prompts, BS)
    ids = _decode_ids(m, kv1, prompts, tables, nxt, BS)
    ref = d1.float().argmax(1)
    top = d1.float().max(1).values
    pick = d1.float().gather(1, ids[:, None])[:, 0]
    assert ((top - pick) <= 2e-2 * top.abs().clamp_min(1)).all()
    assert (ids == ref).float().mean().item() > 0.95


def _decode_ids(m, kv, prompts, tables, next_tok, BS):
    from docqa_amd.models.llama import AttnMeta

    B = len(prompts)
    maxb = max(len(t) for t in tables)
    bt = torch.zeros(B, maxb, dtype=torch.int32)
    for i, t in enumerate(tables):
        bt[i, :len(t)] = torch.tensor(t)
    lens = [len(p) for p in prompts]
    slots = [tables[i][lens[i] // BS] * BS + lens[i] % BS for i in range(B)]
    meta = AttnMeta(prefill=False, positions=torch.tensor(lens, dtype=torch.int32, device="cuda"),
                    slot_mapping=torch.tensor(slots, dtype=torch.int32, device="cuda"),
                    block_tables=bt.cuda(),
                    context_lens=torch.tensor([n + 1 for n in lens], dtype=torch.int32, device="cuda"),
                    max_context=maxb * BS)
    return m.forward(torch.tensor(next_tok, dtype=torch.int32, device="cuda"), meta, kv, greedy_ids=True)


def _mixed_metas(prompts, tables, chunk_prompts, chunk_tables, starts, BS):
    """(decode-step metadata of ``prompts`` -- one new token each after their prompt --,
    prefill metadata of the chunks ``chunk_prompts[i][starts[i]:]`` over their cached heads)."""
    from docqa_amd.models.llama import AttnMeta

    B = len(prompts)
    maxb = max(len(t) for t in tables)
    bt = torch.zeros(B, maxb, dtype=torch.int32)
    for i, t in enumerate(tables):
        bt[i, :len(t)] = torch.tensor(t)
    lens = [len(p) for p in prompts]
    dmeta = AttnMeta(prefill=False, positions=torch.tensor(lens, dtype=torch.int32, device="cuda"),
                     slot_mapping=torch.tensor([tables[i][lens[i] // BS] * BS + lens[i] % BS for i in range(B)],
                                               dtype=torch.int32, device="cuda"),
                     block_tables=bt.cuda(),
                     context_lens=torch.tensor([n + 1 for n in lens], dtype=torch.int32, device="cuda"),
                     max_context=maxb * BS)
    pos, slots, cu = [], [], [0]
    for p, t, s0 in zip(chunk_prompts, chunk_tables, starts):
        pos += list(range(s0, len(p)))
        slots += [t[i // BS] * BS + i % BS for i in range(s0, len(p))]
        cu.append(cu[-1] + len(p) - s0)
    mb = max(len(t) for t in chunk_tables)
    cbt = torch.zeros(len(chunk_tables), mb, dtype=torch.int32)
    for i, t in enumerate(chunk_tables):
        cbt[i, :len(t)] = torch.tensor(t)
    pmeta = AttnMeta(prefill=True, positions=torch.tensor(pos, dtype=torch.int32, device="cuda"),
                     slot_mapping=torch.tensor(slots, dtype=torch.int32, device="cuda"),
                     cu_seqlens=torch.tensor(cu, dtype=torch.int32, device="cuda"),
                     max_len=max(len(p) - s0 for p, s0 in zip(chunk_prompts, starts)),
                     block_tables=cbt.cuda(), prefix_lens=torch.tensor(starts, dtype=torch.int32, device="cuda"))
    return dmeta, pmeta, cu


def test_forward_mixed_native_vs_reference(native):
    """a mixed step -- running decode rows AND prompt chunks in one forward
    (LlamaModel.forward_mixed: every projection over all rows on the prefill GEMMs, attention
    split by row kind, chunks attending their cached heads) -- on the HIP kernels against the
    same step on the fp32 reference ops: logits of every decode row and of each chunk's last
    token (teacher forcing), and the greedy pick wherever the reference's top-2 margin exceeds
    the measured error."""
    from docqa_amd.engine.kv_cache import KVCache
    from docqa_amd.models.llama import LlamaConfig, LlamaModel

    m = LlamaModel(LlamaConfig.preset("llama3-1b-test"), device="cuda", seed=12)
    g = torch.Generator().manual_seed(13)
    BS = 64
    running = [torch.randint(0, 32000, (int(n),), generator=g).tolist() for n in (37, 150, 64, 201)]
    # two new prompts: one from its start, one whose first 128 tokens are already cached
    newp = [torch.randint(0, 32000, (n,), generator=g).tolist() for n in (90, 300)]
    starts = [0, 128]
    nxt = torch.randint(0, 32000, (len(running),), generator=g).tolist()
    out = {}
    for ref in (False, True):
        kv = KVCache(m.cfg.layers, 64, m.hkv, m.cfg.head_dim, BS).caches
        ctx = native.use_reference() if ref else torch.no_grad()
        with ctx:
            _, tables = _prefill_logits(m, kv, running, BS)
            base = sum(len(t) for t in tables)
            ctab = [list(range(base, base + 3)), list(range(base + 3, base + 9))]
            # the cached head of the second new prompt
            _prefill_into(m, kv, newp[1][:starts[1]], ctab[1], BS)
            dmeta, pmeta, cu = _mixed_metas(running, tables, newp, ctab, starts, BS)
            ids = torch.tensor(nxt + [t for p, s0 in zip(newp, starts) for t in p[s0:]], dtype=torch.int32,
                               device="cuda")
            rows = list(range(len(running))) + [len(running) + c - 1 for c in cu[1:]]
            out[ref] = m.forward_mixed(ids, len(running), dmeta, pmeta, kv, torch.tensor(rows, device="cuda"),
                                       return_logits=True).float()
    a, b = out[False], out[True]
    err = _rel(a, b)
    assert err < 0.03, err
    top2 = b.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 4 * err * b.abs().max()
    assert torch.equal(a.argmax(1)[clear], b.argmax(1)[clear])


def _prefill_into(m, kv, prompt, table, BS):
    """Prefill one prompt into the given blocks (its K/V land in the cache)."""
    from docqa_amd.models.llama import AttnMeta

    n = len(prompt)
    meta = AttnMeta(prefill=True, positions=torch.arange(n, dtype=torch.int32, device="cuda"),
                    slot_mapping=torch.tensor([table[t // BS] * BS + t % BS for t in range(n)], dtype=torch.int32,
                                              device="cuda"),
                    cu_seqlens=torch.tensor([0, n], dtype=torch.int32, device="cuda"), max_len=n)
    m.forward(torch.tensor(prompt, dtype=torch.int32, device="cuda"), meta, kv,
              torch.tensor([n - 1], device="cuda"))


def test_llama_graph_vs_eager(native, monkeypatch):
    monkeypatch.setenv("DOCQA_TUNE_DECODE", "0")  # same GEMM kernels on both paths
    from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
    from docqa_amd.models.llama import LlamaConfig, LlamaModel

    m = LlamaModel(LlamaConfig.preset("llama3-1b-test"), device="cuda", seed=3)
    g = torch.Generator().manual_seed(2)
    prompts = [torch.randint(0, 32000, (n,), generator=g).tolist() for n in (40, 77, 5)]
    sp = SamplingParams(max_new_tokens=16, stop_on_eos=False)
    a = LLMEngine(m, max_batch=4, max_context=256, use_graphs=True).generate(prompts, sp)
    b = LLMEngine(m, max_batch=4, max_context=256, use_graphs=False).generate(prompts, sp)
    assert a == b


def test_llama_batch_invariance_logits(native):
    """A prompt's prefill+decode logits are the same alone and inside a batch (paging and
    varlen packing correctness)."""
    from docqa_amd.engine.kv_cache import KVCache
    from docqa_amd.models.llama import LlamaConfig, LlamaModel

    m = LlamaModel(LlamaConfig.preset("llama3-1b-test"), device="cuda", seed=5)
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, 32000, (n,), generator=g).tolist() for n in (50, 200, 3, 90)]
    BS = 64
    kv = KVCache(m.cfg.layers, 64, m.hkv, m.cfg.head_dim, BS).caches
    pb, tb = _prefill_logits(m, kv, prompts, BS)
    db = _decode_logits(m, kv, prompts, tb, [11, 12, 13, 14], BS)
    for i, p in enumerate(prompts):
        kv1 = KVCache(m.cfg.layers, 16, m.hkv, m.cfg.head_dim, BS).caches
        ps, ts = _prefill_logits(m, kv1, [p], BS)
        ds = _decode_logits(m, kv1, [p], ts, [11 + i], BS)
        assert _rel(ps[0], pb[i]) < 0.02
        assert _rel(ds[0], db[i]) < 0.02


@pytest.mark.parametrize("preset", ["llama3-1b-test"])
def test_llama_batch1_decode_xn(native, monkeypatch, preset):
    """Batch-1 decode with the gate|up and next-QKV projections building their own input row
    (residual add + RMSNorm in-kernel, ping-pong residual) == the same step with separate
    add_rmsnorm launches, bit for bit; both track the fp32 reference."""
    from docqa_amd import ops
    from docqa_amd.engine.kv_cache import KVCache
    from docqa_amd.models.llama import LlamaConfig, LlamaModel

    m = LlamaModel(LlamaConfig.preset(preset), device="cuda", seed=11)
    assert ops.xn_ok(1, m.cfg.hidden)
    g = torch.Generator().manual_seed(6)
    V = m.cfg.vocab_size
    prompt = [torch.randint(0, V, (300,), generator=g).tolist()]
    BS = 64
    out = {}
    for xn in (True, False):
        monkeypatch.setattr(ops, "_XN", xn)
        kv = KVCache(m.cfg.layers, 16, m.hkv, m.cfg.head_dim, BS).caches
        _, tb = _prefill_logits(m, kv, prompt, BS)
        out[xn] = _decode_logits(m, kv, prompt, tb, [7], BS)
    assert torch.equal(out[True], out[False])
    with native.use_reference():
        kv = KVCache(m.cfg.layers, 16, m.hkv, m.cfg.head_dim, BS).caches
        _, tb = _prefill_logits(m, kv, prompt, BS)
        ref = _decode_logits(m, kv, prompt, tb, [7], BS)
    assert _rel(out[True], ref) < 0.03


def test_engine_greedy_matches_argmax_of_logits(native):
    """The engine's first generated token is the argmax of the prefill logits."""
    from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
    from docqa_amd.engine.kv_cache import KVCache
    from docqa_amd.models.llama import LlamaConfig, LlamaModel

    m = LlamaModel(LlamaConfig.preset("llama3-1b-test"), device="cuda", seed=9)
    g = torch.Generator().manual_seed(4)
    prompts = [torch.randint(0, 32000, (n,), generator=g).tolist() for n in (33, 70)]
    kv = KVCache(m.cfg.layers, 16, m.hkv, m.cfg.head_dim, 64).caches
    logits, _ = _prefill_logits(m, kv, prompts, 64)
    out = LLMEngine(m, max_batch=2, max_context=256).generate(prompts, SamplingParams(max_new_tokens=2, stop_on_eos=False))
    assert [o[0] for o in out] == logits.float().argmax(-1).tolist()


def test_continuous_engine_graphs(native, monkeypatch):
    """Continuous batching on the GPU with HIP graphs over slot views: simultaneous
    arrivals reproduce the static engine exactly; staggered arrivals (bucket changes,
    slot compaction, more requests than slots) all complete with every block returned."""
    monkeypatch.setenv("DOCQA_TUNE_DECODE", "0")
    from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
    from docqa_amd.engine.scheduler import ContinuousEngine
    from docqa_amd.models.llama import LlamaConfig, LlamaModel

    m = LlamaModel(LlamaConfig.preset("llama3-1b-test"), device="cuda", seed=21)
    g = torch.Generator().manual_seed(5)
    prompts = [torch.randint(3, 32000, (n,), generator=g).tolist() for n in (40, 77, 5, 130)]
    sp = SamplingParams(max_new_tokens=12, stop_on_eos=False)
    static = LLMEngine(m, max_batch=4, max_context=512, use_graphs=True, prefix_cache=False).generate(prompts, sp)
    eng = LLMEngine(m, max_batch=4, max_context=512, use_graphs=True, prefix_cache=False)
    ce = ContinuousEngine(eng)
    assert ce.generate(prompts, sp) == static
    more = [torch.randint(3, 32000, (int(n),), generator=g).tolist() for n in (30, 9, 64, 100, 17, 3, 44)]
    futs = []
    for i, p in enumerate(more):
        futs.append(ce.submit(p, SamplingParams(max_new_tokens=3 + 2 * i, stop_on_eos=False)))
        ce.step()
    while ce.has_work():
        ce.step()
    assert [len(f.result()) for f in futs] == [3 + 2 * i for i in range(len(more))]
    assert len({k[0] for k in ce._graphs}) >= 2      # the batch moved between buckets
    if eng.tail is not None:
        eng.tail.clear()   # blocks pinned by the token-granular prefix cache
    assert eng.kv.allocator.num_free() == eng.kv.num_blocks


def test_checkpoint_roundtrip_generates_identically(native, tmp_path):
    """A model saved as a Hugging Face checkpoint and loaded back onto the GPU (lazy
    safetensors, gate|up re-interleaved for the fused decode GEMM) generates the same
    greedy tokens through the HIP-graph engine."""
    from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
    from docqa_amd.models import checkpoint as ck
    from docqa_amd.models.llama import LlamaConfig, LlamaModel

    m = LlamaModel(LlamaConfig.preset("llama3-1b-test"), device="cuda", seed=11)
    ck.save_llama(m, tmp_path / "ckpt")
    m2 = ck.load_llama(tmp_path / "ckpt", device="cuda")
    g = torch.Generator().manual_seed(5)
    prompts = [torch.randint(0, 32000, (n,), generator=g).tolist() for n in (40, 90, 17)]
    sp = SamplingParams(max_new_tokens=8, stop_on_eos=False)
    a = LLMEngine(m, max_batch=4, max_context=256).generate(prompts, sp)
    b = LLMEngine(m2, max_batch=4, max_context=256).generate(prompts, sp)
    assert a == b


def test_token_classifier_fused_head_matches_unfused(native, monkeypatch):
    """NER predict (fused head+argmax kernel) == F.linear + argmax on the same hidden states."""
    monkeypatch.setenv("DOCQA_NER_FUSED", "1")
    from docqa_amd.deid.engine import NER_LABELS
    from docqa_amd.models.bert import BertConfig, BertTokenClassifier, pack

    clf = BertTokenClassifier(BertConfig.preset("clinical-bert"), NER_LABELS, device="cuda", seed=3)
    assert clf.cls_w.shape[0] == 16
    g = torch.Generator().manual_seed(0)
    toks = [torch.randint(1000, 20000, (n,), generator=g).tolist() for n in (7, 130, 256, 33)]
    ids, cu, max_len = pack(toks, clf.cfg.max_seq_len, clf.device)
    got = clf.predict_packed(ids, cu, max_len)
    with torch.inference_mode():
        h = clf.hidden_states(ids, cu, max_len)
        logits = (h.float() @ clf.cls_w[:len(NER_LABELS)].float().t()
                  + clf.cls_b[:len(NER_LABELS)].float())
    top2 = logits.topk(2, dim=-1).values
    clear = (top2[:, 0] - top2[:, 1]) > 1e-3
    assert got.shape == (ids.numel(),)
    assert torch.equal(got[clear].cpu(), logits.argmax(-1)[clear].cpu())
    assert clear.float().mean().item() > 0.95


def test_grouped_decode_without_common_prefix(native, monkeypatch):
    """Batches whose rows share no prompt prefix (the reference QA template) take the
    grouped split-plan decode with the prefix attended inline (LLMEngine.group_without_prefix)
    instead of the per-row ring kernel: same generations up to fp summation-order near-ties."""
    from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
    from docqa_amd.models.llama import LlamaConfig, LlamaModel

    m = LlamaModel(LlamaConfig.preset("llama3-1b-test"), device="cuda", seed=31)
    g = torch.Generator().manual_seed(8)
    shared = [torch.randint(3, 32000, (int(n),), generator=g).tolist() for n in (70, 150)]
    prompts = []
    for i in range(40):      # some rows share a retrieved "chunk" after a unique head, none share a prefix
        head = torch.randint(3, 32000, (5 + i % 7,), generator=g).tolist()
        prompts.append(head + shared[i % 2] + torch.randint(3, 32000, (20 + 3 * i,), generator=g).tolist())
    sp = SamplingParams(max_new_tokens=10, stop_on_eos=False)
    outs = {}
    for flag in (False, True):
        eng = LLMEngine(m, max_batch=64, max_context=512, use_graphs=True)
        eng.group_without_prefix = (lambda B, f=flag, e=eng, orig=LLMEngine.group_without_prefix:
                                    f and orig(e, B))
        assert LLMEngine.group_without_prefix(eng, 40) or not flag
        outs[flag] = eng.generate(prompts, sp)
    # random-init logits are nearly flat, so a summation-order difference flips a greedy
    # pick now and then (~3 % of tokens) and the sequence diverges from there: compare the
    # first decode step's tokens (one attention pass per layer on identical inputs)
    first = sum(a[1] == b[1] for a, b in zip(outs[False], outs[True]))
    assert first >= 0.9 * len(prompts), first
    assert [o[0] for o in outs[True]] == [o[0] for o in outs[False]]          # prefill: same path
    assert all(len(o) == 10 for o in outs[True])
