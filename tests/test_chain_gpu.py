"""Persistent decode-layer chain (csrc/kernels/mgemm.hip mgemm_chain_kernel): O -> add+RMSNorm
-> gate|up+SwiGLU -> down -> add+RMSNorm -> next QKV in one launch.  It runs the standalone
kernels' tiles and norm rows as work items, so its outputs must equal the six-launch
sequence BIT FOR BIT (and track the fp32 PyTorch reference of the block); its counters must
come back zeroed (graph replays need no memset) with no lost wake-up flagged."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def native():
    from docqa_amd import ops

    assert ops.load_native(build_if_missing=True), "native extension failed to load"
    return ops


def _layer(H, Ko, inter, Nq, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)

    def w(n, k):
        return (torch.randn(n, k, device="cuda", generator=g) / k ** 0.5).bfloat16()

    return dict(o=w(H, Ko), gate_up=w(2 * inter, H), down=w(H, inter), qkv=w(Nq, H),
                post=(1 + 0.1 * torch.randn(H, device="cuda", generator=g)).bfloat16(),
                nxt=(1 + 0.1 * torch.randn(H, device="cuda", generator=g)).bfloat16())


def _sequence(ops, a, L, residual, plan, eps, with_qkv=True):
    """The six standalone launches the chain replaces (llama.py decode, TP = 1)."""
    S_o, c_o, S_d, c_d, S_q, c_q = plan
    nat = torch.ops.docqa
    x1 = nat.add_rmsnorm_splitk(nat.mgemm(a, L["o"], S_o, c_o), residual, L["post"], eps)
    g = nat.mgemm_glu(x1, L["gate_up"], 2)
    x2 = nat.add_rmsnorm_splitk(nat.mgemm(g, L["down"], S_d, c_d), residual, L["nxt"], eps)
    pq = nat.mgemm(x2, L["qkv"], S_q, c_q) if with_qkv else None
    return x2, pq


@pytest.fixture
def chain_on(native, monkeypatch):
    monkeypatch.setattr(native, "_CHAIN", True)
    return native


# Llama-3-8B decode shapes (O 64-wide tiles, down S=7), a 2-m-tile bucket and tail rows;
# the 1B-test layer (every split-K phase on 64-wide tiles)
@pytest.mark.parametrize("M,H,Ko,inter,Nq", [(256, 4096, 4096, 14336, 6144), (512, 4096, 4096, 14336, 6144),
                                             (200, 4096, 4096, 14336, 6144), (256, 2048, 2048, 8192, 3072)])
def test_chain_matches_sequence(chain_on, M, H, Ko, inter, Nq):
    ops = chain_on
    plan = ops.chain_plan(M, H, Ko, 2 * inter, Nq)
    assert plan is not None, "the chain should apply at this shape"
    L = _layer(H, Ko, inter, Nq)
    a = torch.randn(M, Ko, device="cuda").bfloat16()
    res0 = torch.randn(M, H, device="cuda").bfloat16()
    eps = 1e-5
    r_seq = res0.clone()
    x2_seq, pq_seq = _sequence(ops, a, L, r_seq, plan, eps)
    ctr = torch.zeros(16, dtype=torch.int32, device="cuda")
    for it in range(3):   # a publish/acquire race would show up intermittently; counters reset
        r = res0.clone()
        x2, pq = ops.mgemm_chain(a, L["o"], r, L["post"], L["gate_up"], L["down"], L["nxt"], L["qkv"], ctr, plan,
                                 eps)
        torch.cuda.synchronize()
        assert int(ctr[12]) == 0, "lost wake-up flagged"
        assert int(ctr[:10].abs().sum()) == 0, f"counters not reset: {ctr.tolist()}"
        assert torch.equal(r, r_seq), f"residual differs (iteration {it})"
        assert torch.equal(x2, x2_seq), f"x2 differs (iteration {it})"
        assert torch.equal(pq, pq_seq), f"QKV slabs differ (iteration {it})"
    # and the block itself against fp32 PyTorch
    rf = res0.float() + (a.float() @ L["o"].float().T)
    x1 = rf * torch.rsqrt(rf.pow(2).mean(-1, keepdim=True) + eps) * L["post"].float()
    gu = x1 @ L["gate_up"].float().T
    gu = gu.view(M, -1, 2, 8)          # 8-interleaved gate | up rows
    gl = (torch.nn.functional.silu(gu[:, :, 0]) * gu[:, :, 1]).reshape(M, inter)
    rf = rf + gl @ L["down"].float().T
    x2f = rf * torch.rsqrt(rf.pow(2).mean(-1, keepdim=True) + eps) * L["nxt"].float()
    err = (x2.float() - x2f).abs().max().item()
    assert err < 0.1 * x2f.abs().max().item(), err


def test_chain_last_layer_and_graph_replay(chain_on):
    """No next QKV (last layer), captured once in a HIP graph and replayed: every replay
    starts from the counters the previous one reset."""
    ops = chain_on
    M, H, Ko, inter, Nq = 256, 4096, 4096, 14336, 6144
    plan = ops.chain_plan(M, H, Ko, 2 * inter, Nq)
    L = _layer(H, Ko, inter, Nq, seed=1)
    a = torch.randn(M, Ko, device="cuda").bfloat16()
    res0 = torch.randn(M, H, device="cuda").bfloat16()
    ctr = torch.zeros(16, dtype=torch.int32, device="cuda")
    r = res0.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):   # warm-up outside capture
        ops.mgemm_chain(a, L["o"], r, L["post"], L["gate_up"], L["down"], L["nxt"], None, ctr, plan, 1e-5)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        x2, pq = ops.mgemm_chain(a, L["o"], r, L["post"], L["gate_up"], L["down"], L["nxt"], None, ctr, plan, 1e-5)
    assert pq is None
    for _ in range(3):
        r.copy_(res0)
        graph.replay()
        torch.cuda.synchronize()
        r_seq = res0.clone()
        x2_seq, _ = _sequence(ops, a, L, r_seq, plan, 1e-5, with_qkv=False)
        assert int(ctr[12]) == 0 and int(ctr[:10].abs().sum()) == 0
        assert torch.equal(x2, x2_seq) and torch.equal(r, r_seq)


def test_llama_decode_chain_token_exact(chain_on, monkeypatch):
    """A decode forward of the 1B-test model at a 256-row bucket: chain on == chain off."""
    from docqa_amd.models.llama import AttnMeta, LlamaConfig, LlamaModel

    ops = chain_on
    cfg = LlamaConfig.preset("llama3-1b-test")
    model = LlamaModel(cfg, device="cuda", seed=3)
    B, ctx, bs = 256, 96, 64
    nblk = (ctx + bs - 1) // bs
    kv = [(torch.randn(B * nblk + 1, cfg.kv_heads, bs, cfg.head_dim, device="cuda").bfloat16(),
           torch.randn(B * nblk + 1, cfg.kv_heads, bs, cfg.head_dim, device="cuda").bfloat16())
          for _ in range(cfg.layers)]
    tables = (torch.arange(B * nblk, device="cuda", dtype=torch.int32).view(B, nblk) + 1)
    pos = torch.full((B,), ctx - 1, device="cuda", dtype=torch.int32)
    slots = tables[:, (ctx - 1) // bs] * bs + (ctx - 1) % bs
    meta = AttnMeta(prefill=False, positions=pos, slot_mapping=slots.int(), block_tables=tables,
                    context_lens=torch.full((B,), ctx, device="cuda", dtype=torch.int32), max_context=ctx)
    ids = torch.randint(0, cfg.vocab_size, (B,), device="cuda", dtype=torch.int32)

    def run(on):
        monkeypatch.setattr(ops, "_CHAIN", on)
        caches = [(k.clone(), v.clone()) for k, v in kv]
        return model.forward(ids, meta, caches, greedy_ids=True), model.forward(ids, meta, caches)

    ids_on, logits_on = run(True)
    ids_off, logits_off = run(False)
    assert torch.equal(ids_on, ids_off)
    assert torch.equal(logits_on, logits_off)
