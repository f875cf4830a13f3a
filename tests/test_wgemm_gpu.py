"""Mid-M decode GEMM with the weights streamed into VGPRs (csrc/kernels/wgemm.hip) against
the fp32 PyTorch reference: bf16 output, split-K fp32 slabs, fused SwiGLU (1 slice, and 2
K halves meeting in the launch), fused LM-head argmax.  ``cfg``: wgemm.hip variant."""
import pytest
import torch

pytestmark = pytest.mark.gpu
CFGS = [1, 2, 3, 4, 9]


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


@pytest.mark.parametrize("M", [1, 193, 256, 300])
@pytest.mark.parametrize("N,K,S", [(6144, 4096, 8), (4096, 4096, 16), (4096, 14336, 14), (1024, 1024, 1),
                                   (1024, 1024, 2), (512, 192, 1), (768, 2048, 4)])
@pytest.mark.parametrize("cfg", CFGS)
def test_wgemm(native, M, N, K, S, cfg):
    bn = torch.ops.docqa.wgemm_tile_n(cfg)
    if N % bn:
        pytest.skip("N not a multiple of the tile")
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    ref = x.float() @ w.float().T
    for _ in range(3):   # a ring-pipeline race would show up intermittently
        out = torch.ops.docqa.wgemm(x, w, S, cfg)
        if S == 1:
            assert out.shape == (M, N) and out.dtype == torch.bfloat16
            _close(out, ref, 2e-2, 1e-2)
        else:
            assert out.shape == (S, M, N) and out.dtype == torch.float32
            _close(out.sum(0), ref, 2e-3, 1e-3)


@pytest.mark.parametrize("cfg", CFGS)
def test_wgemm_asymmetric_identity(native, cfg):
    """X = I rows against an asymmetric W: catches transposed / mis-placed tile writes."""
    M, N, K = 256, 512, 1024
    x = torch.zeros(M, K, device="cuda", dtype=torch.bfloat16)
    x[torch.arange(M), torch.arange(M) * 3] = 1
    w = (torch.arange(N * K, device="cuda").view(N, K) % 97).bfloat16()
    want = w.float()[:, torch.arange(M, device="cuda") * 3].T
    assert torch.equal(torch.ops.docqa.wgemm(x, w, 1, cfg).float(), want)
    assert torch.equal(torch.ops.docqa.wgemm(x, w, 4, cfg).sum(0), want)


def _glu_ws(M, N, cfg):
    bn = torch.ops.docqa.wgemm_tile_n(cfg)
    mt = (M + 255) // 256
    ws = torch.empty(mt * N * 256, device="cuda", dtype=torch.float32)
    tick = torch.zeros(2 * mt * (N // bn) + 1, device="cuda", dtype=torch.int32)
    return ws, tick


@pytest.mark.parametrize("M", [200, 256, 333])
@pytest.mark.parametrize("S", [1, 2])
@pytest.mark.parametrize("cfg", CFGS)
def test_wgemm_glu(native, M, S, cfg):
    from docqa_amd.ops import reference as R

    N, K = 28672, 4096
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    ref = R.silu_mul((x.float() @ w.float().T).bfloat16(), interleaved=True)
    ws, tick = _glu_ws(M, N, cfg)
    outs = []
    for _ in range(3):   # the hand-off words must re-arm between launches
        out = torch.ops.docqa.wgemm_glu(x, w, S, cfg, ws, tick)
        _close(out, ref, 2e-2, 1e-2)
        outs.append(out)
    assert int(tick.abs().sum()) == 0, "tickets / error word not re-armed"
    # which K half parks its partial varies; fp32 a + b == b + a keeps the bits identical
    assert all(torch.equal(outs[0], o) for o in outs[1:])


def test_wgemm_glu_graph_replay(native):
    """The 2-way hand-off inside a captured graph: tickets re-arm across replays."""
    from docqa_amd.ops import reference as R

    M, N, K, cfg = 256, 2048, 1024, 1
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    ws, tick = _glu_ws(M, N, cfg)
    ref = R.silu_mul((x.float() @ w.float().T).bfloat16(), interleaved=True)
    torch.ops.docqa.wgemm_glu(x, w, 2, cfg, ws, tick)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = torch.ops.docqa.wgemm_glu(x, w, 2, cfg, ws, tick)
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    _close(out, ref, 2e-2, 1e-2)
    assert int(tick.abs().sum()) == 0


@pytest.mark.parametrize("M", [1, 256, 300])
@pytest.mark.parametrize("cfg", [1, 3])
def test_wgemm_argmax(native, M, cfg):
    """LM head + greedy pick == argmax of the bf16 logits (ties: lowest id)."""
    N, K = 128256, 4096
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    logits = (x.float() @ w.float().T).bfloat16().float()
    n_valid = N - 100
    ids, vals = torch.ops.docqa.wgemm_argmax_val(x, w, n_valid, cfg)
    want = logits[:, :n_valid].argmax(1)
    got_v = logits.gather(1, ids[:, None])[:, 0]
    # exact ties in bf16 are legal either way only when values are equal
    assert torch.equal(got_v, logits.gather(1, want[:, None])[:, 0])
    assert torch.equal(vals, got_v)
    assert int(ids.max()) < n_valid


@pytest.mark.parametrize("cfg", [17, 18, 20, 25])
@pytest.mark.parametrize("N,K,S", [(6144, 4096, 8), (4096, 14336, 14), (1024, 1024, 2)])
def test_wgemm_packed_weights(native, cfg, N, K, S):
    """Fragment-major packed weights (ops.pack_fragments): same product as row-major."""
    from docqa_amd import ops

    bn = torch.ops.docqa.wgemm_tile_n(cfg)
    if N % bn:
        pytest.skip("N not a multiple of the tile")
    M = 256
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    wp = ops.pack_fragments(w)
    ref = x.float() @ w.float().T
    _close(torch.ops.docqa.wgemm(x, wp, S, cfg).sum(0), ref, 2e-3, 1e-3)
    _close(torch.ops.docqa.wgemm(x, wp, 1, cfg), ref, 2e-2, 1e-2)


@pytest.mark.parametrize("cfg", [17, 18])
def test_wgemm_packed_glu_and_argmax(native, cfg):
    from docqa_amd import ops
    from docqa_amd.ops import reference as R

    M, N, K = 256, 28672, 4096
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    wp = ops.pack_fragments(w)
    ref = R.silu_mul((x.float() @ w.float().T).bfloat16(), interleaved=True)
    ws, tick = _glu_ws(M, N, cfg)
    for S in (1, 2):
        _close(torch.ops.docqa.wgemm_glu(x, wp, S, cfg, ws, tick), ref, 2e-2, 1e-2)
    logits = (x.float() @ w.float().T).bfloat16().float()
    ids, vals = torch.ops.docqa.wgemm_argmax_val(x, wp, N, cfg)
    assert torch.equal(logits.gather(1, ids[:, None])[:, 0], logits.max(1).values)
