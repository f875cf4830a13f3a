"""Stream-K mid-M GEMM (mgemm.hip mgemm_sk_kernel): a persistent grid splits the (tile, K
unit) iterations evenly; tiles cut between workgroups are finished in-launch by the last
arriving piece.  Checked against a plain PyTorch fp32 reference of the same op, for bf16,
fused SwiGLU and fp32-slab epilogues, row counts that are not multiples of 256, grids that
cut tiles into 1..5 pieces -- and bit-for-bit determinism (the pieces are summed in K order
whoever arrives last)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ws(M, N, K, grid):
    nat = torch.ops.docqa
    part = torch.empty(nat.mgemm_sk_part_floats(grid), device="cuda")
    cnt = torch.zeros(2 * ((M + 255) // 256) * (N // 128), dtype=torch.int32, device="cuda")
    return part, cnt


@pytest.mark.parametrize("M,N,K,grid", [(256, 1024, 1024, 0), (600, 2048, 2048, 0), (768, 4096, 1024, 37),
                                        (1000, 1280, 4096, 0), (200, 768, 2048, 5), (513, 2048, 1536, 256)])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_stream_k_matches_fp32_reference(M, N, K, grid, epi):
    from docqa_amd import ops

    assert ops.load_native()
    nat = torch.ops.docqa
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    G = nat.mgemm_sk_grid(M, N, K, grid or cus)
    assert 1 <= G <= (grid or cus)
    part, cnt = _ws(M, N, K, G)
    out = nat.mgemm_sk(x, w, epi, part, cnt, G)
    ref = x.float() @ w.float().t()
    if epi == 1:
        from docqa_amd.ops import reference as R

        ref = R.silu_mul(ref.to(torch.bfloat16).float(), interleaved=True).float()
        assert out.shape == (M, N // 2)
        torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=3e-2)
    elif epi == 2:
        assert out.shape == (1, M, N) and out.dtype == torch.float32
        torch.testing.assert_close(out[0], ref, atol=2e-3 * float(ref.abs().max()), rtol=1e-3)
    else:
        torch.testing.assert_close(out.float(), ref, atol=2e-2 * float(ref.abs().max()) ** 0.5, rtol=2e-2)
    assert int(cnt.abs().sum()) == 0                      # every ticket re-armed
    again = nat.mgemm_sk(x, w, epi, part, cnt, G)
    assert torch.equal(out, again)                        # K-order sums: bit-for-bit repeatable


def test_stream_k_grid_bounds_pieces_per_tile():
    nat = torch.ops.docqa
    from docqa_amd import ops

    assert ops.load_native()
    # 1 tile of 32 units on 256 CUs: at most 5 pieces -> grid <= 5 (8 units each, 4 pieces)
    assert nat.mgemm_sk_grid(256, 128, 4096, 256) <= 5
    assert nat.mgemm_sk_grid(768, 6144, 4096, 256) == 256
