"""Batch-1 register-streaming GEMV (dgemm.hip gemv_kernel) against the fp32 reference: split-K
slabs at every (rows per workgroup, split) it is instantiated for, the SwiGLU epilogue over
8-interleaved gate|up rows, the in-kernel input row (residual add + RMSNorm of the previous
projection's slabs) against the ring kernel's identical prologue, and a batch-1 decode of
the Llama test preset on the GEMV plans against the reference forward."""
import pytest
import torch

from docqa_amd import ops
from docqa_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    assert ops.load_native(build_if_missing=True)
    return ops


def _w(N, K, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) / K ** 0.5).to(torch.bfloat16)


@pytest.mark.parametrize("N,K,S,R", [(6144, 4096, 2, 4), (4096, 4096, 1, 8), (1024, 2048, 1, 16),
                                     (512, 8192, 2, 8), (256, 14336, 7, 4), (4096, 14336, 1, 4)])
def test_gemv_slabs_match_fp32(N, K, S, R):
    assert ops.load_native()
    x = (torch.rand(1, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = _w(N, K, 1)
    P = torch.ops.docqa.gemv(x, w, S, R, False)
    assert P.shape == (S, 1, N) and P.dtype == torch.float32
    r = x.float() @ w.float().t()
    assert (P.sum(0) - r).abs().max().item() <= 1e-3 * r.abs().max().item() + 1e-4


@pytest.mark.parametrize("N,K", [(28672, 4096), (2048, 2048), (512, 4096)])
def test_gemv_glu_matches_fp32(N, K):
    assert ops.load_native()
    x = (torch.rand(1, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = _w(N, K, 2)
    y = torch.ops.docqa.gemv(x, w, 1, 16, True)
    r = ref.silu_mul((x.float() @ w.float().t()).bfloat16(), interleaved=True).float()
    assert y.shape == (1, N // 2)
    assert (y.float() - r).abs().max().item() <= 2e-2 * r.abs().max().item() + 1e-3


@pytest.mark.parametrize("glu", [False, True])
def test_gemv_xn_matches_ring_prologue(glu):
    """Same input-row arithmetic as dgemm_partial_xn / dgemm_glu_xn: same residual out,
    products equal up to the dot-product order."""
    assert ops.load_native()
    H, N = 4096, (28672 if glu else 6144)
    g = torch.Generator(device="cuda").manual_seed(3)
    Pin = torch.randn(3, 1, H, device="cuda", generator=g)
    res = torch.randn(1, H, device="cuda", generator=g).to(torch.bfloat16)
    gamma = (1 + 0.1 * torch.randn(H, device="cuda", generator=g)).to(torch.bfloat16)
    w = _w(N, H, 4)
    r1, r2 = torch.empty_like(res), torch.empty_like(res)
    if glu:
        a = ops.gemv_glu_xn(Pin, res, r1, gamma, 1e-5, w)
        b = ops.dgemm_glu_xn(Pin, res, r2, gamma, 1e-5, w)
    else:
        a = ops.gemv_partial_xn(Pin, res, r1, gamma, 1e-5, w, 1, 8).sum(0)
        b = ops.dgemm_partial_xn(Pin, res, r2, gamma, 1e-5, w, 2).sum(0)
    assert torch.equal(r1, r2)
    assert (a.float() - b.float()).abs().max().item() <= 1e-2 * b.float().abs().max().item() + 1e-3


def test_llama_batch1_decode_on_gemv_plans(native):
    """One-row decode steps of the Llama test preset take the GEMV plans (QKV / O slabs,
    SwiGLU gate|up with the in-kernel input row) and track the fp32 reference forward."""
    from docqa_amd.engine.kv_cache import KVCache
    from docqa_amd.models.llama import LlamaConfig, LlamaModel
    from tests.test_models_gpu import _decode_logits, _prefill_logits, _rel

    m = LlamaModel(LlamaConfig.preset("llama3-1b-test"), device="cuda", seed=17)
    L0 = m.layers[0]
    assert ops.gemv_plan(1, *L0["qkv"].shape)[0] and ops.gemv_glu_ok(1, *L0["gate_up"].shape)
    prompts = [torch.randint(0, 32000, (77,), generator=torch.Generator().manual_seed(5)).tolist()]
    BS = 64
    kv1 = KVCache(m.cfg.layers, 16, m.hkv, m.cfg.head_dim, BS).caches
    kv2 = KVCache(m.cfg.layers, 16, m.hkv, m.cfg.head_dim, BS).caches
    _, tables = _prefill_logits(m, kv1, prompts, BS)
    d1 = _decode_logits(m, kv1, prompts, tables, [4], BS)
    with native.use_reference():
        _prefill_logits(m, kv2, prompts, BS)
        d2 = _decode_logits(m, kv2, prompts, tables, [4], BS)
    assert _rel(d1, d2) < 0.03


@pytest.mark.parametrize("N,K,n_valid", [(128256, 4096, 128256), (32000, 2048, 31990), (4096, 4096, 1000)])
def test_gemv_argmax_matches_bf16_logits(N, K, n_valid):
    """Batch-1 LM head + greedy pick on the GEMV == argmax of the bf16 fp32-accumulated
    logits over the valid vocabulary (ties to the lowest id), planted winner included."""
    assert ops.load_native()
    x = (torch.rand(1, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = _w(N, K, 5)
    w[n_valid - 1] = (x.float() * 4).to(torch.bfloat16)[0]     # a clear winner at the last valid id
    if n_valid < N:
        w[n_valid] = (x.float() * 8).to(torch.bfloat16)[0]     # past n_valid: must be ignored
    ids, vals = torch.ops.docqa.gemv_argmax_val(x, w, n_valid)
    logits = (x.float() @ w[:n_valid].float().t()).bfloat16().float()
    assert int(ids[0]) == int(logits.argmax(1)[0]) == n_valid - 1
    assert abs(float(vals[0]) - float(logits.max())) <= 1e-2 * abs(float(logits.max()))
    assert int(ops.lm_head_argmax(x, w, n_valid)[0]) == n_valid - 1
