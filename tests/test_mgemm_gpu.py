"""Mid-M decode GEMM (csrc/kernels/mgemm.hip, 193..512-row decode buckets) against the fp32
PyTorch reference: bf16 output, split-K fp32 slabs, fused SwiGLU, fused LM-head argmax.
``cfg``: the kernel variant (tile width / stage depth / wave layout, mgemm.hip kCfg)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def native():
    from docqa_amd import ops

    assert ops.load_native(build_if_missing=True), "native extension failed to load"
    torch.manual_seed(0)
    return ops


def _close(a, b, atol, rtol=0.0):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"max err {err} > {tol}"


@pytest.mark.parametrize("M", [1, 100, 193, 256, 300, 512])
@pytest.mark.parametrize("N,K,S,bn", [(6144, 4096, 4, 2), (4096, 4096, 8, 4), (4096, 14336, 7, 1),
                                      (4096, 14336, 8, 3), (1024, 1024, 1, 2), (1024, 1024, 2, 4),
                                      (512, 128, 1, 4), (768, 2048, 16, 1), (768, 3072, 4, 3),
                                      (6144, 4096, 8, 3), (512, 64, 1, 3), (6144, 4096, 8, 5), (4096, 14336, 14, 6),
                                      (1024, 1024, 1, 5), (512, 128, 1, 6), (768, 1024, 2, 6),
                                      (4096, 4096, 4, 7), (4096, 14336, 7, 7), (6144, 4096, 2, 7), (64, 128, 1, 7)])
def test_mgemm(native, M, N, K, S, bn):
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    ref = x.float() @ w.float().T
    for _ in range(3):   # a ring-pipeline race would show up intermittently
        out = torch.ops.docqa.mgemm(x, w, S, bn)
        if S == 1:
            assert out.shape == (M, N) and out.dtype == torch.bfloat16
            _close(out, ref, 2e-2, 1e-2)
        else:
            assert out.shape == (S, M, N) and out.dtype == torch.float32
            _close(out.sum(0), ref, 2e-3, 1e-3)


@pytest.mark.parametrize("bn", [1, 2, 3, 4, 5, 6, 7])
def test_mgemm_asymmetric_identity(native, bn):
    """X = I rows against an asymmetric W: catches transposed / mis-placed tile writes."""
    M, N, K = 256, 512, 1024
    x = torch.zeros(M, K, device="cuda", dtype=torch.bfloat16)
    x[torch.arange(M), torch.arange(M) * 3] = 1
    w = (torch.arange(N * K, device="cuda").view(N, K) % 97).bfloat16()
    o = torch.ops.docqa.mgemm(x, w, 1, bn).float()
    assert torch.equal(o, w.float()[:, torch.arange(M, device="cuda") * 3].T)
    P = torch.ops.docqa.mgemm(x, w, 4, bn)
    assert torch.equal(P.sum(0), w.float()[:, torch.arange(M, device="cuda") * 3].T)


@pytest.mark.parametrize("M", [200, 256, 333])
@pytest.mark.parametrize("bn", [1, 2, 3, 4, 5, 6])
def test_mgemm_glu(native, M, bn):
    from docqa_amd.ops import reference as R

    N, K = 28672, 4096
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    ref = R.silu_mul((x.float() @ w.float().T).bfloat16(), interleaved=True)
    for _ in range(2):
        _close(torch.ops.docqa.mgemm_glu(x, w, bn), ref, 2e-2, 1e-2)


@pytest.mark.parametrize("M", [1, 256, 300])
@pytest.mark.parametrize("bn", [1, 2, 3, 4, 5, 6])
def test_mgemm_argmax(native, M, bn):
    """LM head + greedy pick == argmax of the bf16 logits (ties: lowest id)."""
    N, K = 128256, 4096
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    logits = (x.float() @ w.float().T)
    got = torch.ops.docqa.mgemm_argmax(x, w, N, bn)
    assert got.dtype == torch.long and got.shape == (M,)
    # the fp32-accumulated logit of the chosen id must equal the row max within bf16
    # rounding (accumulation order differs from torch's)
    top = logits.max(1).values
    pick = logits.gather(1, got[:, None])[:, 0]
    assert ((top - pick) <= 2e-2 * top.abs().clamp_min(1)).all()
    agree = (got == logits.bfloat16().float().argmax(1)).float().mean().item()
    assert agree > 0.97
    # vocabulary padding excluded: n_valid masks the tail columns
    w2 = w.clone()
    w2[-128:] = w2[-128:] * 0 + 1
    x2 = x.abs()
    got2 = torch.ops.docqa.mgemm_argmax(x2, w2, N - 128, bn)
    assert (got2 < N - 128).all()


def test_mgemm_glu_rejects_narrow_tiles(native):
    """cfg 7 (64-wide tiles) has no SwiGLU epilogue: refused, not silently wrong."""
    x = torch.randn(256, 4096, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(1024, 4096, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        torch.ops.docqa.mgemm_glu(x, w, 7)


def test_mgemm_argmax_ties(native):
    """Every logit equal: the lowest index wins (torch.argmax tie rule)."""
    M, N, K = 256, 2048, 512
    x = torch.ones(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.full((N, K), 0.5, device="cuda", dtype=torch.bfloat16)
    assert (torch.ops.docqa.mgemm_argmax(x, w, N, 2) == 0).all()
    assert (torch.ops.docqa.mgemm_argmax(x, w, N, 6) == 0).all()
    w[700:] = 0.75
    w[1500] = 1.0
    assert (torch.ops.docqa.mgemm_argmax(x, w, N, 4) == 1500).all()
    assert (torch.ops.docqa.mgemm_argmax(x, w, N, 6) == 1500).all()
    w[1500] = 0.75
    w[1999] = 1.0       # the best id in the last 256-column tile, beside the n_valid mask
    assert (torch.ops.docqa.mgemm_argmax(x, w, N, 6) == 1999).all()
    assert (torch.ops.docqa.mgemm_argmax(x, w, 1999, 6) == 700).all()
