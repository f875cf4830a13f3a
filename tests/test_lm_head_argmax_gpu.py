"""LM head + greedy pick with the argmax fused into the decode GEMM at every bucket
(VERDICT r3 missing #2 / next #4): dgemm.hip EPI_ARGMAX at <= 192 rows (batch-1 decode
included), mgemm.hip at 193..512 -- against the argmax of the fp32-reference logits
rounded to bf16 (ties: lowest id)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def native():
    from docqa_amd import ops

    assert ops.load_native(build_if_missing=True)
    torch.manual_seed(0)
    return ops


@pytest.fixture(scope="module")
def head():
    N, K = 128256, 4096
    return (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()


def _check(x, w, ids, vals, n_valid):
    logits = (x.float() @ w.float().T).bfloat16().float()[:, :n_valid]
    want = logits.argmax(1)
    got_v = logits.gather(1, ids[:, None])[:, 0]
    assert torch.equal(got_v, logits.gather(1, want[:, None])[:, 0])
    assert torch.equal(vals, got_v)
    assert int(ids.max()) < n_valid


@pytest.mark.parametrize("M", [1, 3, 16, 33, 64, 100, 128, 150, 192])
def test_dgemm_argmax(native, head, M):
    x = torch.randn(M, head.shape[1], device="cuda", dtype=torch.bfloat16)
    n_valid = head.shape[0] - 256
    ids, vals = torch.ops.docqa.dgemm_argmax_val(x, head, n_valid)
    _check(x, head, ids, vals, n_valid)


@pytest.mark.parametrize("M", [1, 64, 192, 193, 256, 300])
def test_lm_head_argmax_dispatch_every_bucket(native, head, M):
    """ops.lm_head_argmax takes the fused path at every row count 1..512."""
    from docqa_amd import ops

    assert ops.lm_head_argmax_ok(M, *head.shape)
    x = torch.randn(M, head.shape[1], device="cuda", dtype=torch.bfloat16)
    ids, vals = ops.lm_head_argmax(x, head, head.shape[0], with_values=True)
    _check(x, head, ids, vals, head.shape[0])
