"""bf16 split-K slabs (DOCQA_SLAB_BF16): the mid-M decode GEMM's EPI_PARTIAL16 epilogue
(csrc/kernels/mgemm.hip) and its two consumers -- RoPE + paged-cache write
(rope_cache.hip) and residual add + RMSNorm (norm.hip / docqa_norm_row.h) -- against a
plain PyTorch fp32 reference of the same ops, and bit-exact against the fp32-slab consumers
fed the same bf16-rounded partials."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def native():
    from docqa_amd import ops

    assert ops.load_native(build_if_missing=True), "native extension failed to load"
    torch.manual_seed(0)
    return ops


@pytest.mark.parametrize("M", [193, 256, 300])
@pytest.mark.parametrize("N,K,S,cfg", [(6144, 4096, 4, 2), (4096, 4096, 4, 7), (4096, 14336, 8, 2),
                                       (1024, 1024, 2, 6)])
def test_mgemm_slab16(native, M, N, K, S, cfg):
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    P16 = torch.ops.docqa.mgemm_slab16(x, w, S, cfg)
    assert P16.shape == (S, M, N) and P16.dtype == torch.bfloat16
    # every slab is the fp32 slab rounded once to bf16
    P32 = torch.ops.docqa.mgemm(x, w, S, cfg)
    assert torch.equal(P16, P32.bfloat16())
    ref = x.float() @ w.float().T
    err = (P16.float().sum(0) - ref).abs().max().item()
    assert err <= 2e-2 + 1e-2 * ref.abs().max().item()


def test_add_rmsnorm_splitk16(native):
    S, M, H = 8, 256, 4096
    P16 = (torch.randn(S, M, H, device="cuda") * 0.3).bfloat16()
    res = torch.randn(M, H, device="cuda").bfloat16()
    g = (1 + 0.1 * torch.randn(H, device="cuda")).bfloat16()
    r16, r32 = res.clone(), res.clone()
    o16 = native.add_rmsnorm_splitk(P16, r16, g, 1e-5)
    o32 = native.add_rmsnorm_splitk(P16.float(), r32, g, 1e-5)
    assert torch.equal(o16, o32) and torch.equal(r16, r32)
    # fp32 reference of the op
    x = (P16.float().sum(0).bfloat16().float() + res.float()).bfloat16().float()
    ref = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * g.float()
    assert (r16.float() - x).abs().max().item() == 0.0
    assert (o16.float() - ref).abs().max().item() < 5e-2


def test_rope_cache_splitk16(native):
    S, T, Hq, Hkv, D, BS = 4, 256, 32, 8, 128, 64
    P16 = torch.randn(S, T, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
    pos = torch.randint(0, 2000, (T,), device="cuda", dtype=torch.int32)
    inv = 1.0 / (500000.0 ** (torch.arange(0, D, 2, device="cuda").float() / D))
    ang = torch.arange(4096, device="cuda").float()[:, None] * inv[None]
    cos_sin = torch.cat([ang.cos(), ang.sin()], -1).contiguous()
    nblocks = T // BS + 2
    slots = torch.randperm(nblocks * BS, device="cuda")[:T].int()
    kc16 = torch.zeros(nblocks, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)
    vc16 = torch.zeros_like(kc16)
    kc32, vc32 = kc16.clone(), vc16.clone()
    q16 = native.rope_cache_splitk(P16, pos, cos_sin, slots, kc16, vc16, Hq, Hkv, D)
    q32 = native.rope_cache_splitk(P16.float(), pos, cos_sin, slots, kc32, vc32, Hq, Hkv, D)
    assert torch.equal(q16, q32) and torch.equal(kc16, kc32) and torch.equal(vc16, vc32)
    # fp32 reference: rotate-half RoPE of bf16(sum of slabs)
    x = P16.float().sum(0).bfloat16().float().view(T, Hq + 2 * Hkv, D)
    c = cos_sin[pos.long(), : D // 2][:, None]
    s = cos_sin[pos.long(), D // 2:][:, None]
    qk = x[:, : Hq + Hkv]
    x1, x2 = qk[..., : D // 2], qk[..., D // 2:]
    rot = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1)
    assert (q16.float().view(T, -1, D)[:, : Hq + Hkv] - rot).abs().max().item() < 5e-2
    assert torch.equal(q16.view(T, -1, D)[:, Hq + Hkv:].float(), x[:, Hq + Hkv:])


@pytest.mark.parametrize("M", [193, 256])
def test_glu_split16(native, M):
    """Batch-256 gate|up on 256-wide tiles split over K into bf16 slabs + the bf16 split-K
    SwiGLU consumer, against the fp32 reference and bit-exact against the fp32-slab consumer
    fed the same bf16 partials."""
    K, I = 4096, 14336
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(2 * I, K, device="cuda") / K ** 0.5).bfloat16()
    P16 = torch.ops.docqa.mgemm_slab16(x, w, 2, 6)
    o16 = torch.ops.docqa.silu_mul_splitk(P16)
    o32 = torch.ops.docqa.silu_mul_splitk(P16.float())
    assert torch.equal(o16, o32)
    assert torch.equal(native.glu_split16(x, w, 2, 6), o16)
    gu = (x.float() @ w.float().T).view(M, -1, 2, 8)
    ref = (torch.nn.functional.silu(gu[:, :, 0]) * gu[:, :, 1]).reshape(M, I)
    err = (o16.float() - ref).abs().max().item()
    assert err <= 3e-2 + 2e-2 * ref.abs().max().item()
