"""Grouped cascade decode (attn_decode.hip paged_decode_group_kernel): rows that share
prefix-cache KV blocks are attended together in groups of <= 4; the result must equal the
per-row cascade decode and the fp32 reference for any packing of the rows."""
import math
import random

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def native():
    from docqa_amd import ops

    assert ops.load_native(build_if_missing=True)
    torch.manual_seed(0)
    return ops


def _trie_batch(B, P_blocks, maxb, seed):
    """Block tables with a common prefix of P_blocks and clusters of rows sharing 1-4 more
    blocks (a prefix-cache trie), then unique blocks; context lengths past the prefix."""
    rnd = random.Random(seed)
    nxt = P_blocks
    prefix = list(range(P_blocks))
    tables, lens = [], []
    while len(tables) < B:
        csize = rnd.choice([1, 1, 2, 3, 5])
        depth = rnd.randint(0, 4)
        shared = list(range(nxt, nxt + depth))
        nxt += depth
        for _ in range(min(csize, B - len(tables))):
            own = list(range(nxt, nxt + maxb - P_blocks - depth))
            nxt += len(own)
            tables.append(prefix + shared + own)
            lens.append(64 * (P_blocks + depth) + rnd.randint(1, 64 * 3))
    return tables, lens, nxt


@pytest.mark.parametrize("B,Hkv,seed", [(37, 8, 0), (64, 2, 1), (5, 8, 2), (256, 8, 3)])
def test_grouped_cascade_matches_per_row(native, B, Hkv, seed):
    from docqa_amd.ops import reference as R

    Hq, D, BS, Pb, maxb = 4 * Hkv, 128, 64, 3, 12
    tables, lens, nblk = _trie_batch(B, Pb, maxb, seed)
    kc = torch.randn(nblk, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.tensor(tables, dtype=torch.int32, device="cuda")
    cl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    pt = torch.zeros(maxb, dtype=torch.int32, device="cuda")
    pt[:Pb] = bt[0, :Pb]
    plen = torch.tensor([Pb * BS], dtype=torch.int32, device="cuda")
    scale = 1 / math.sqrt(D)
    ref = native.paged_decode_cascade(q, kc, vc, bt, cl, Hq, maxb * BS, scale, pt, plen, 4)
    with native.use_reference():
        ref32 = native.paged_decode_cascade(q, kc, vc, bt, cl, Hq, maxb * BS, scale, pt, plen, 4)
    cap = (B + 1) // 2
    for packing in ("trie", "consecutive", "reversed"):
        if packing == "trie":
            quads = native.pack_decode_groups(tables, lens, Pb, BS, cap)
        elif packing == "consecutive":
            quads = [list(range(i, min(B, i + 4))) for i in range(0, B, 4)]
        else:
            rows = list(range(B))[::-1]
            quads = [rows[i:i + 3] for i in range(0, B, 3)]
        assert sorted(r for qd in quads for r in qd) == list(range(B))
        flat = torch.full((max(cap, len(quads)) * 4,), -1, dtype=torch.int32)
        for i, qd in enumerate(quads):
            flat[4 * i:4 * i + len(qd)] = torch.tensor(qd, dtype=torch.int32)
        out = native.paged_decode_cascade_grouped(q, kc, vc, bt, cl, Hq, scale, pt, plen, 4, flat.cuda())
        err = (out.float() - ref.float()).abs().max().item()
        assert err < 2e-2, (packing, err)
        err32 = (out.float() - ref32.float()).abs().max().item()
        assert err32 < 3e-2, (packing, err32)


def test_grouped_cascade_padded_rows_zero(native):
    """Rows with no keys past the prefix (padded decode slots) get zeros."""
    Hkv, D, BS, Pb, maxb = 2, 128, 64, 2, 6
    Hq, B = 4 * Hkv, 6
    tables, lens, nblk = _trie_batch(B, Pb, maxb, 7)
    lens[2] = 0
    lens[5] = Pb * BS
    kc = torch.randn(nblk, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.tensor(tables, dtype=torch.int32, device="cuda")
    cl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    pt = bt[0].clone()
    plen = torch.tensor([Pb * BS], dtype=torch.int32, device="cuda")
    groups = torch.tensor([0, 1, 2, 3, 4, 5, -1, -1], dtype=torch.int32, device="cuda")
    out = native.paged_decode_cascade_grouped(q, kc, vc, bt, cl, Hq, 1 / math.sqrt(D), pt, plen, 2, groups)
    assert torch.isfinite(out.float()).all()
    assert (out[2] == 0).all() and (out[5] == 0).all()


@pytest.mark.parametrize("B,Hkv,seed", [(37, 8, 0), (256, 8, 3), (9, 2, 5)])
@pytest.mark.parametrize("tiles", [1, 3, 12, 1000])
@pytest.mark.parametrize("defer", [False, True])
def test_split_grouped_cascade_matches_per_row(native, B, Hkv, seed, tiles, defer):
    """Split plan (long groups over several workgroups + LSE merge) == per-row cascade and
    the fp32 reference; planned with END-of-decode lengths longer than the current ones,
    so some items have no keys yet.  ``defer``: every group merged by the merge kernel and
    the prefix kernel forked onto a side stream."""
    Hq, D, BS, Pb, maxb = 4 * Hkv, 128, 64, 3, 12
    tables, lens, nblk = _trie_batch(B, Pb, maxb, seed)
    kc = torch.randn(nblk, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.tensor(tables, dtype=torch.int32, device="cuda")
    cl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    pt = torch.zeros(maxb, dtype=torch.int32, device="cuda")
    pt[:Pb] = bt[0, :Pb]
    plen = torch.tensor([Pb * BS], dtype=torch.int32, device="cuda")
    scale = 1 / math.sqrt(D)
    ref = native.paged_decode_cascade(q, kc, vc, bt, cl, Hq, maxb * BS, scale, pt, plen, 4)
    with native.use_reference():
        ref32 = native.paged_decode_cascade(q, kc, vc, bt, cl, Hq, maxb * BS, scale, pt, plen, 4)
    end_lens = [min(L + 128, maxb * BS) for L in lens]
    quads = native.pack_decode_groups(tables, end_lens, Pb, BS, (B + 1) // 2)
    plan = native.split_decode_groups(quads, tables, end_lens, Pb, BS, max(B, 4), tiles, defer=defer)
    if tiles == 1:
        assert (plan[1, :, 5] > 1).any()   # some group really is split
    if defer:
        assert (plan[0, :, 6][plan[0, :, 0] >= 0] >= 0).all()   # every item writes a partial
    out = native.paged_decode_cascade_grouped(q, kc, vc, bt, cl, Hq, scale, pt, plen, 4, plan.cuda(), defer)
    err = (out.float() - ref.float()).abs().max().item()
    assert err < 2e-2, err
    err32 = (out.float() - ref32.float()).abs().max().item()
    assert err32 < 3e-2, err32
    if not defer:
        # inline prefix: items from block 0 (plan built with skip 0), the groups attend the
        # shared prefix themselves -- no prefix kernel -- same attention
        quads0 = native.pack_decode_groups(tables, end_lens, Pb, BS, (B + 1) // 2)
        plan0 = native.split_decode_groups(quads0, tables, end_lens, 0, BS, max(B, 4), tiles)
        o0 = native.paged_decode_cascade_grouped(q, kc, vc, bt, cl, Hq, scale, pt, plen, 4, plan0.cuda(), False,
                                                 None, True)
        err0 = (o0.float() - ref32.float()).abs().max().item()
        assert err0 < 3e-2, err0
        # split groups merged by their last item (ticket words, no merge launch) == the
        # merge kernel, with the tickets re-armed after every launch
        tick = torch.zeros(plan.shape[1] * Hkv, dtype=torch.int32, device="cuda")
        for _ in range(2):
            o2 = native.paged_decode_cascade_grouped(q, kc, vc, bt, cl, Hq, scale, pt, plen, 4, plan.cuda(),
                                                     False, tick)
            torch.cuda.synchronize()
            d = (o2.float() - out.float()).abs()
            bad = (d > 0).any(1).nonzero().flatten().tolist()
            print(f"tick merge vs merge kernel: max |diff| {d.max().item():.3g}, rows {bad[:16]} of {len(bad)}")
            # same fold order; the two merge instantiations may contract a multiply-add
            # differently: bf16 rounding-level differences only (a stale partial would not be)
            assert d.max().item() <= 2e-3 + 1e-2 * out.float().abs().max().item(), d.max().item()
            assert int(tick.abs().sum()) == 0


@pytest.mark.parametrize("B,Hkv,seed,S", [(37, 8, 0, 4), (256, 8, 3, 4), (9, 2, 5, 1), (64, 8, 6, 2)])
@pytest.mark.parametrize("tiles", [3, 12])
def test_grouped_fused_matches_unfused(native, B, Hkv, seed, S, tiles):
    """Grouped decode straight from QKV split-K slabs (RoPE + new-token cache write inside the
    group kernel) == rope_cache_splitk + the inline-prefix grouped kernel: same output and
    the same cache contents."""
    Hq, D, BS, Pb, maxb = 4 * Hkv, 128, 64, 3, 12
    tables, lens, nblk = _trie_batch(B, Pb, maxb, seed)
    lens = [max(L, 1) for L in lens]
    kc = torch.randn(nblk, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.tensor(tables, dtype=torch.int32, device="cuda")
    cl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    pos = cl - 1
    slots = (bt.gather(1, (pos // BS).long()[:, None])[:, 0] * BS + pos % BS).int()
    if B > 4:
        slots[3] = -1                       # a row without a cache write
    P = torch.randn(S, B, (Hq + 2 * Hkv) * D, device="cuda") * 0.5
    cs = native.reference.rope_cos_sin(maxb * BS, D, 500000.0, "cuda")
    pt = torch.zeros(maxb, dtype=torch.int32, device="cuda")
    pt[:Pb] = bt[0, :Pb]
    plen = torch.tensor([Pb * BS], dtype=torch.int32, device="cuda")
    scale = 1 / math.sqrt(D)
    end_lens = [min(L + 128, maxb * BS) for L in lens]
    quads = native.pack_decode_groups(tables, end_lens, Pb, BS, (B + 1) // 2)
    plan = native.split_decode_groups(quads, tables, end_lens, 0, BS, max(B, 4), tiles).cuda()
    kc1, vc1, kc2, vc2 = kc.clone(), vc.clone(), kc.clone(), vc.clone()
    qkv = native.rope_cache_splitk(P, pos, cs, slots, kc1, vc1, Hq, Hkv, D)
    ref = native.paged_decode_cascade_grouped(qkv, kc1, vc1, bt, cl, Hq, scale, pt, plen, 4, plan, False, None, True)
    tick = torch.zeros(plan.shape[1] * Hkv, dtype=torch.int32, device="cuda")
    got = native.paged_decode_grouped_fused(P, pos, cs, slots, kc2, vc2, bt, cl, Hq, scale, pt, plen, 4, plan, tick)
    torch.cuda.synchronize()
    assert torch.equal(kc2, kc1) and torch.equal(vc2, vc1)
    d = (got.float() - ref.float()).abs().max().item()
    assert d <= 2e-3 + 1e-2 * ref.float().abs().max().item(), d
    assert int(tick.abs().sum()) == 0


def test_split_grouped_cascade_padded_rows_zero(native):
    Hkv, D, BS, Pb, maxb = 2, 128, 64, 2, 6
    Hq, B = 4 * Hkv, 6
    tables, lens, nblk = _trie_batch(B, Pb, maxb, 7)
    plan = native.split_decode_groups([[0, 1, 2], [3, 4, 5]], tables, [maxb * BS] * B, Pb, BS, 8, 1)
    lens[2] = 0
    lens[5] = Pb * BS
    kc = torch.randn(nblk, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.tensor(tables, dtype=torch.int32, device="cuda")
    cl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    pt = bt[0].clone()
    plen = torch.tensor([Pb * BS], dtype=torch.int32, device="cuda")
    out = native.paged_decode_cascade_grouped(q, kc, vc, bt, cl, Hq, 1 / math.sqrt(D), pt, plen, 2, plan.cuda())
    tick = torch.zeros(8 * Hkv, dtype=torch.int32, device="cuda")
    o2 = native.paged_decode_cascade_grouped(q, kc, vc, bt, cl, Hq, 1 / math.sqrt(D), pt, plen, 2, plan.cuda(),
                                             False, tick)
    assert (o2.float() - out.float()).abs().max().item() <= 2e-3 and int(tick.abs().sum()) == 0
    assert torch.isfinite(out.float()).all()
    assert (out[2] == 0).all() and (out[5] == 0).all()
    assert (out[0].float().abs().sum() > 0) and (out[4].float().abs().sum() > 0)


@pytest.mark.parametrize("B,Hkv,seed", [(37, 8, 0), (256, 8, 3), (9, 2, 5), (512, 8, 4)])
@pytest.mark.parametrize("tiles", [1, 3, 12, 1000])
def test_persistent_grouped_cascade_matches_per_row(native, B, Hkv, seed, tiles):
    """Persistent plan (work items packed into bins, one ring per workgroup across item
    boundaries, every group merged) == per-row cascade and the fp32 reference; END-of-decode
    planning lengths, so some items have no live keys yet."""
    Hq, D, BS, Pb, maxb = 4 * Hkv, 128, 64, 3, 12
    tables, lens, nblk = _trie_batch(B, Pb, maxb, seed)
    kc = torch.randn(nblk, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.tensor(tables, dtype=torch.int32, device="cuda")
    cl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    pt = torch.zeros(maxb, dtype=torch.int32, device="cuda")
    pt[:Pb] = bt[0, :Pb]
    plen = torch.tensor([Pb * BS], dtype=torch.int32, device="cuda")
    scale = 1 / math.sqrt(D)
    ref = native.paged_decode_cascade(q, kc, vc, bt, cl, Hq, maxb * BS, scale, pt, plen, 4)
    with native.use_reference():
        ref32 = native.paged_decode_cascade(q, kc, vc, bt, cl, Hq, maxb * BS, scale, pt, plen, 4)
    end_lens = [min(L + 128, maxb * BS) for L in lens]
    cap = max(B, 4)
    quads = native.pack_decode_groups(tables, end_lens, Pb, BS, (B + 1) // 2)
    nb = native.persist_bins(cap, Hkv)
    assert nb == torch.ops.docqa.group_persist_bins(cap, Hkv)
    plan = native.split_decode_groups(quads, tables, end_lens, Pb, BS, cap, tiles, bins=nb)
    assert plan.shape == (3, cap, 8)
    used = plan[2][plan[2] >= 0]
    assert used.numel() == int((plan[0, :, 6] >= 0).sum())          # every item in one bin
    out = native.paged_decode_cascade_grouped(q, kc, vc, bt, cl, Hq, scale, pt, plen, 4, plan.cuda())
    err = (out.float() - ref.float()).abs().max().item()
    assert err < 2e-2, err
    err32 = (out.float() - ref32.float()).abs().max().item()
    assert err32 < 3e-2, err32


@pytest.mark.parametrize("mode", ["persist", "defer", "split"])
def test_identity_plan_matches_per_row(native, monkeypatch, mode):
    """The engine's identity plan (consecutive quads, before set_groups runs) in each plan
    mode: persistent (one quad per bin), deferred (every quad merged, prefix forked) and
    plain split (quads finish in their workgroup)."""
    from docqa_amd.engine.llm_engine import _defer_groups_on, _identity_groups

    monkeypatch.setenv("DOCQA_GROUP_PERSIST", "1" if mode == "persist" else "0")
    monkeypatch.setenv("DOCQA_GROUP_DEFER", "1" if mode == "defer" else "0")

    Hkv, D, BS, Pb, maxb, B = 8, 128, 64, 2, 10, 64
    Hq = 4 * Hkv
    tables, lens, nblk = _trie_batch(B, Pb, maxb, 11)
    kc = torch.randn(nblk, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.tensor(tables, dtype=torch.int32, device="cuda")
    cl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    pt = torch.zeros(maxb, dtype=torch.int32, device="cuda")
    pt[:Pb] = bt[0, :Pb]
    plen = torch.tensor([Pb * BS], dtype=torch.int32, device="cuda")
    scale = 1 / math.sqrt(D)
    plan = _identity_groups(B, "cuda", Hkv)
    assert plan.shape[0] == (3 if mode == "persist" else 2)
    ref = native.paged_decode_cascade(q, kc, vc, bt, cl, Hq, maxb * BS, scale, pt, plen, 4)
    out = native.paged_decode_cascade_grouped(q, kc, vc, bt, cl, Hq, scale, pt, plen, 4, plan,
                                              _defer_groups_on())
    assert (out.float() - ref.float()).abs().max().item() < 2e-2


@pytest.mark.parametrize("B,Hkv,seed,maxb", [(37, 8, 0, 12), (256, 8, 3, 12), (9, 2, 5, 12), (12, 8, 7, 64)])
@pytest.mark.parametrize("tiles", [1, 3, 12, 1000])
@pytest.mark.parametrize("inline", [False, True])
@pytest.mark.parametrize("variant", [1, 2, 3, 4])
def test_wave_kernel_matches_cooperative(native, B, Hkv, seed, maxb, tiles, inline, variant):
    """attn_decode.hip paged_decode_group_wave_kernel in each shape (waves x ring slots: 4 x 2,
    2 x 3, 2 x 4, 1 x 4; each wave streams its own 16-token quarter tiles through a private
    ring; per-wave states combined once) == the cooperative
    split kernel and the fp32 reference: cascade prefix kernel or inline prefix, ticket merges
    re-armed, END-of-decode planning lengths, up to 64 block positions per row."""
    Hq, D, BS, Pb = 4 * Hkv, 128, 64, 3
    tables, lens, nblk = _trie_batch(B, Pb, maxb, seed)
    if maxb == 64:   # long rows: most of the 64 block positions live
        rnd = random.Random(seed)
        lens = [min(64 * maxb - 128, L + 64 * rnd.randint(20, 58)) for L in lens]
    kc = torch.randn(nblk, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.tensor(tables, dtype=torch.int32, device="cuda")
    cl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    pt = torch.zeros(maxb, dtype=torch.int32, device="cuda")
    pt[:Pb] = bt[0, :Pb]
    plen = torch.tensor([Pb * BS], dtype=torch.int32, device="cuda")
    scale = 1 / math.sqrt(D)
    with native.use_reference():
        ref32 = native.paged_decode_cascade(q, kc, vc, bt, cl, Hq, maxb * BS, scale, pt, plen, 4)
    end_lens = [min(L + 128, maxb * BS) for L in lens]
    quads = native.pack_decode_groups(tables, end_lens, Pb, BS, (B + 1) // 2)
    plan = native.split_decode_groups(quads, tables, end_lens, 0 if inline else Pb, BS, max(B, 4), tiles).cuda()
    tick = torch.zeros(plan.shape[1] * Hkv, dtype=torch.int32, device="cuda")
    was = torch.ops.docqa.set_group_wave(0)
    try:
        coop = native.paged_decode_cascade_grouped(q, kc, vc, bt, cl, Hq, scale, pt, plen, 4, plan, False, tick,
                                                   inline)
        torch.ops.docqa.set_group_wave(variant)
        for _ in range(2):
            wave = native.paged_decode_cascade_grouped(q, kc, vc, bt, cl, Hq, scale, pt, plen, 4, plan, False,
                                                       tick, inline)
            torch.cuda.synchronize()
            assert int(tick.abs().sum()) == 0
            err32 = (wave.float() - ref32.float()).abs().max().item()
            assert err32 < 3e-2, err32
            d = (wave.float() - coop.float()).abs().max().item()
            assert d < 2e-2, d
    finally:
        torch.ops.docqa.set_group_wave(was)


@pytest.mark.parametrize("variant", [0, 1])
def test_remapped_plan_after_retirement_matches_per_row(native, variant):
    """Requests retire and the survivors are compacted: the plan re-targeted by
    ops.remap_plan_rows (no re-plan) still gives the per-row attention of the survivors,
    with the merge tickets left re-armed (fully retired groups draw none)."""
    Hkv, D, BS, Pb, maxb, B = 8, 128, 64, 3, 12, 96
    Hq = 4 * Hkv
    tables, lens, nblk = _trie_batch(B, Pb, maxb, 21)
    end_lens = [min(L + 128, maxb * BS) for L in lens]
    quads = native.pack_decode_groups(tables, end_lens, Pb, BS, (B + 1) // 2)
    plan = native.split_decode_groups(quads, tables, end_lens, 0, BS, B, 3)
    ids = list(range(1000, 1000 + B))
    rnd = random.Random(3)
    keep = sorted(rnd.sample(range(B), 80))
    for qd in quads[:3]:                         # retire three whole groups too
        keep = [i for i in keep if i not in qd]
    new_plan = native.remap_plan_rows(plan, ids, [ids[i] for i in keep])
    assert new_plan is not None
    assert native.remap_plan_rows(plan, ids, [ids[i] for i in keep] + [7]) is None   # an admission
    tables2, lens2 = [tables[i] for i in keep], [lens[i] for i in keep]
    n = len(keep)
    kc = torch.randn(nblk, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.tensor(tables2, dtype=torch.int32, device="cuda")
    cl = torch.tensor(lens2, dtype=torch.int32, device="cuda")
    q = torch.randn(n, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    pt = torch.zeros(maxb, dtype=torch.int32, device="cuda")
    pt[:Pb] = bt[0, :Pb]
    plen = torch.tensor([Pb * BS], dtype=torch.int32, device="cuda")
    scale = 1 / math.sqrt(D)
    with native.use_reference():
        ref32 = native.paged_decode_cascade(q, kc, vc, bt, cl, Hq, maxb * BS, scale, pt, plen, 4)
    tick = torch.zeros(B * Hkv, dtype=torch.int32, device="cuda")
    was = torch.ops.docqa.set_group_wave(variant)
    try:
        for _ in range(2):
            out = native.paged_decode_cascade_grouped(q, kc, vc, bt, cl, Hq, scale, pt, plen, 4, new_plan.cuda(),
                                                      False, tick, True)
            torch.cuda.synchronize()
            assert int(tick.abs().sum()) == 0
            err = (out.float() - ref32.float()).abs().max().item()
            assert err < 3e-2, err
    finally:
        torch.ops.docqa.set_group_wave(was)


@pytest.mark.parametrize("B,Hkv,seed", [(37, 8, 0), (256, 8, 3)])
@pytest.mark.parametrize("inline", [False, True])
def test_wave_kernel_on_a_wide_block_table(native, B, Hkv, seed, inline):
    """A block table sized for a long MAX_CONTEXT (128 wide: the llm-qa service's 8192
    tokens) with rows that end within 64 blocks (LLMEngine.groups_fit) -- the grouped wave
    kernel gives the result it gives on the same rows in a 64-wide table and matches the
    fp32 reference."""
    Hq, D, BS, Pb, maxb = 4 * Hkv, 128, 64, 3, 12
    tables, lens, nblk = _trie_batch(B, Pb, maxb, seed)
    kc = torch.randn(nblk, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    narrow = torch.tensor([t + [0] * (64 - len(t)) for t in tables], dtype=torch.int32, device="cuda")
    wide = torch.zeros(B, 128, dtype=torch.int32, device="cuda")
    wide[:, :64] = narrow
    wide[:, 64:] = 0              # past every row's end: attending these would change the result
    cl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    plen = torch.tensor([Pb * BS], dtype=torch.int32, device="cuda")
    scale = 1 / math.sqrt(D)
    end_lens = [L + 128 for L in lens]
    quads = native.pack_decode_groups(tables, end_lens, Pb, BS, (B + 1) // 2)
    plan = native.split_decode_groups(quads, tables, end_lens, 0 if inline else Pb, BS, max(B, 4), 12).cuda()
    outs = []
    for bt in (narrow, wide):
        pt = torch.zeros(bt.shape[1], dtype=torch.int32, device="cuda")
        pt[:Pb] = bt[0, :Pb]
        tick = torch.zeros(plan.shape[1] * Hkv, dtype=torch.int32, device="cuda")
        outs.append(native.paged_decode_cascade_grouped(q, kc, vc, bt, cl, Hq, scale, pt, plen, 4, plan, False,
                                                        tick, inline))
        torch.cuda.synchronize()
        assert int(tick.abs().sum()) == 0
    with native.use_reference():
        pt = torch.zeros(64, dtype=torch.int32, device="cuda")
        pt[:Pb] = narrow[0, :Pb]
        ref32 = native.paged_decode_cascade(q, kc, vc, narrow, cl, Hq, 64 * BS, scale, pt, plen, 4)
    assert torch.equal(outs[0], outs[1])
    assert (outs[1].float() - ref32.float()).abs().max().item() < 3e-2
