"""Prefill GEMM (csrc/kernels/pgemm.hip: 256 x 256 x 64 8-phase MFMA schedule, LDS-DMA
half-tiles, staggered wave rows) against the fp32 PyTorch reference of the same op,
bf16 out and the fused SwiGLU epilogue over 8-interleaved gate|up rows."""
import pytest
import torch

from docqa_amd import ops
from docqa_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

SHAPES = [  # (M, N, K): tails in M, one K-tile pair, deep K, Llama-3-8B / 70B-TP8 shapes
    (256, 256, 128), (1, 256, 256), (300, 512, 256), (1000, 1280, 1024), (2048, 6144, 4096),
    (513, 4096, 14336), (4096, 1024, 3584),
]


def _data(M, N, K, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(torch.bfloat16)
    return x, w


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_pgemm_bf16_matches_fp32_reference(M, N, K):
    assert ops.load_native()
    x, w = _data(M, N, K)
    y = torch.ops.docqa.pgemm(x, w, 0)
    r = x.float() @ w.float().t()
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    err = (y.float() - r).abs().max().item()
    assert err <= 2e-2 * r.abs().max().item() + 1e-3, err


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (777, 1024, 512), (2048, 28672 // 8, 4096)])
def test_pgemm_swiglu_epilogue(M, N, K):
    x, w = _data(M, N, K, seed=1)
    y = torch.ops.docqa.pgemm(x, w, 1)
    r = ref.silu_mul((x.float() @ w.float().t()), interleaved=True).float()
    assert y.shape == (M, N // 2)
    err = (y.float() - r).abs().max().item()
    assert err <= 2e-2 * r.abs().max().item() + 1e-3, err


def test_pgemm_asymmetric_exact_small_ints():
    """Integer-valued operands (exact in bf16 and fp32): every output element must be exact,
    which catches a transposed or mis-placed C write that random data might blur."""
    M, N, K = 512, 768, 256
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randint(-3, 4, (M, K), device="cuda", generator=g).to(torch.bfloat16)
    w = torch.randint(-2, 3, (N, K), device="cuda", generator=g).to(torch.bfloat16)
    w[:, 0] = torch.arange(N, device="cuda").remainder(7).to(torch.bfloat16)   # asymmetric in N
    y = torch.ops.docqa.pgemm(x, w, 0).float()
    r = (x.float() @ w.float().t()).to(torch.bfloat16).float()   # exact sums, one rounding
    assert torch.equal(y, r)


def test_prefill_dispatch_routes_to_hand_written_kernels():
    x, w = _data(4096, 4096, 1024, seed=4)
    assert ops.pgemm_ok(4096, 4096, 1024)
    y = ops.prefill_linear(x, w)
    r = x.float() @ w.float().t()
    assert (y.float() - r).abs().max().item() <= 2e-2 * r.abs().max().item()
    xs, ws = _data(40, 384, 256, seed=5)   # few tiles: the 128 x 128 kernel
    ys = ops.prefill_linear(xs, ws)
    rs = xs.float() @ ws.float().t()
    assert (ys.float() - rs).abs().max().item() <= 2e-2 * rs.abs().max().item()


@pytest.mark.parametrize("M,N,K,S", [(256, 6144, 4096, 8), (200, 4096, 14336, 4), (512, 1280, 8192, 16),
                                     (37, 512, 1024, 2), (256, 256, 256, 1)])
def test_pgemm_splitk_slabs(M, N, K, S):
    x, w = _data(M, N, K, seed=6)
    P = torch.ops.docqa.pgemm_partial(x, w, S)
    assert P.shape == (S, M, N) and P.dtype == torch.float32
    r = x.float() @ w.float().t()
    err = (P.sum(0) - r).abs().max().item()
    assert err <= 2e-3 * r.abs().max().item() + 1e-3, err
    # each slab is its own K range
    Ks = K // S
    r0 = x[:, :Ks].float() @ w[:, :Ks].float().t()
    assert (P[0] - r0).abs().max().item() <= 2e-3 * r0.abs().max().item() + 1e-3


@pytest.mark.parametrize("M,N,K", [(512, 7168, 8192), (1000, 7168, 1024), (77, 256, 128)])
def test_gemm128_swiglu_epilogue(M, N, K):
    """gemm.hip EPI_GLU (128 x 128 tiles, SwiGLU over 8-interleaved gate|up rows, inputs
    rounded to bf16 like the unfused GEMM's output) == the fp32 reference; the prefill
    dispatch takes it where the 256-wide tiles leave the chip idle (70B TP-8 gate|up)."""
    x, w = _data(M, N, K, seed=7)
    y = torch.ops.docqa.gemm(x, w, None, None, ops.EPI_GLU)
    r = ref.silu_mul((x.float() @ w.float().t()), interleaved=True).float()
    assert y.shape == (M, N // 2)
    err = (y.float() - r).abs().max().item()
    assert err <= 2e-2 * r.abs().max().item() + 1e-3, err
    y2 = ops.prefill_glu(x, w)
    assert (y2.float() - r).abs().max().item() <= 2e-2 * r.abs().max().item() + 1e-3


def test_prefill_split_plan_slabs_feed_the_consumers():
    """The narrow-N prefill split (ops.prefill_split_plan, the 70B TP-8 QKV shard) picks
    S with tiles x S <= 256 and K % (128 S) == 0; its slabs sum to the product."""
    assert ops.prefill_split_plan(512, 1280, 8192) == 8
    assert ops.prefill_split_plan(4096, 1280, 8192) == 2
    assert ops.prefill_split_plan(512, 6144, 4096) == 0           # wide N: no split
    x, w = _data(700, 1280, 8192, seed=8)
    S = ops.prefill_split_plan(700, 1280, 8192)
    P = ops.pgemm_partial(x, w, S)
    r = x.float() @ w.float().t()
    assert (P.sum(0) - r).abs().max().item() <= 2e-3 * r.abs().max().item() + 1e-3


@pytest.mark.parametrize("M,N,K,glu", [(512, 7168, 8192, True), (600, 8192, 3584, False), (768, 6144, 4096, False),
                                       (1200, 4096, 4096, False), (1024, 4096, 14336, False), (512, 1280, 8192, False),
                                       (300, 4096, 14336, False), (2048, 7168, 8192, True), (700, 28672, 4096, True)])
def test_prefill_route_products(M, N, K, glu):
    """Every route the prefill forward can take (ops.prefill_route: hand-written tiles, split-K
    slabs into the consumers, the SwiGLU split-K consumer) computes the projection: fp32 slabs summed, bf16
    products and SwiGLU outputs against the fp32 reference."""
    x, w = _data(M, N, K, seed=3)
    label, fn = ops.prefill_route(M, N, K, glu=glu, down=(K == 14336 or K == 3584))
    y = fn(x, w)
    if y.dim() == 3:
        y = y.sum(0)
    r = x.float() @ w.float().t()
    if glu:
        r = ref.silu_mul(r.bfloat16(), interleaved=True).float()
    err = (y.float() - r).abs().max().item() / max(1e-6, r.abs().max().item())
    assert y.shape == r.shape, label
    assert err < 2e-2, (label, err)
    assert "hipblaslt" not in label


@pytest.mark.parametrize("S,M,I", [(1, 7, 64), (2, 300, 3584), (4, 512, 3584), (8, 33, 128)])
def test_silu_mul_splitk_matches_reference(S, M, I):
    """The SwiGLU split-K consumer (act.hip silu_mul_splitk): fp32 slabs of an 8-interleaved
    gate|up projection summed in slab order, rounded as the bf16 GEMM output, silu(gate) * up."""
    g = torch.Generator(device="cuda").manual_seed(S * 1000 + M)
    P = torch.randn(S, M, 2 * I, device="cuda", generator=g)
    got = torch.ops.docqa.silu_mul_splitk(P)
    want = ref.silu_mul(P.sum(0).to(torch.bfloat16), interleaved=True).float()
    assert got.shape == (M, I) and got.dtype == torch.bfloat16
    assert (got.float() - want).abs().max().item() <= 2e-2 * want.abs().max().item() + 1e-3


def test_70b_gate_up_split_route_matches_fused_epilogue():
    """The 70B TP-8 gate|up shard at 512 rows takes K-split slabs + silu_mul_splitk (no
    library GEMM): same values as the 256 x 256 kernel's fused SwiGLU epilogue up to the
    K-split summation order."""
    x, w = _data(512, 7168, 8192, seed=11)
    assert ops.prefill_split_plan(512, 7168, 8192, glu=True) == 4
    a = ops.prefill_glu(x, w).float()
    b = torch.ops.docqa.pgemm(x, w, 1).float()
    assert (a - b).abs().max().item() <= 2e-2 * b.abs().max().item() + 1e-3
