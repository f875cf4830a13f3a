"""Token-granular prefix copies (csrc/kernels/rope_cache.hip kv_copy_rows): one launch
copies K/V rows [0, m) of a source block into the same rows of a destination block in
every layer's pools -- bitwise equal to the tensor-indexing reference, rows past m and
other blocks untouched."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def native():
    from docqa_amd import ops

    assert ops.load_native(build_if_missing=True)
    return ops


@pytest.mark.parametrize("Hkv,BS,D", [(8, 64, 128), (2, 16, 64)])
def test_kv_copy_rows_matches_indexing(native, Hkv, BS, D):
    torch.manual_seed(0)
    L, NB = 3, 40
    pools = [(torch.randn(NB, Hkv, BS, D, device="cuda").bfloat16(),
              torch.randn(NB, Hkv, BS, D, device="cuda").bfloat16()) for _ in range(L)]
    ref = [(k.cpu().clone(), v.cpu().clone()) for k, v in pools]
    copies = [(3, 7, 1), (5, 9, BS - 1), (11, 12, BS // 2), (30, 2, 5)]
    native.kv_copy_rows(pools, copies)
    native.kv_copy_rows(ref, copies)          # CPU: tensor indexing
    for (k, v), (rk, rv) in zip(pools, ref):
        assert torch.equal(k.cpu(), rk) and torch.equal(v.cpu(), rv)
    # rows past m of a destination keep their old values (copy 0 moved row 0 only)
    assert torch.equal(ref[0][0][7, :, 1:], pools[0][0][7, :, 1:].cpu())


def test_kv_copy_rows_out_of_range_is_skipped(native):
    pools = [(torch.zeros(4, 1, 16, 64, device="cuda", dtype=torch.bfloat16),
              torch.zeros(4, 1, 16, 64, device="cuda", dtype=torch.bfloat16))]
    pools[0][0][0] = 1
    native.kv_copy_rows(pools, [(0, 9, 4), (0, 1, 99), (0, 2, 3)])   # bad dst / rows: skipped
    torch.cuda.synchronize()
    assert pools[0][0][1].abs().sum() == 0
    assert (pools[0][0][2, :, :3] == 1).all() and (pools[0][0][2, :, 3:] == 0).all()
