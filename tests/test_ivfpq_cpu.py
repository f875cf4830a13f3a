"""IVF-PQ on CPU (reference path): training, residual encoding, inverted lists, ADC
search quality against exact search, incremental adds, FAISS-format round trip."""
import torch

from docqa_amd.index import faiss_io
from docqa_amd.index.flat import FlatIndex
from docqa_amd.index.ivfpq import IVFPQIndex


def _data(n=4000, d=64, seed=0):
    g = torch.Generator().manual_seed(seed)
    c = torch.randn(40, d, generator=g) * 3
    x = c[torch.randint(0, 40, (n,), generator=g)] + torch.randn(n, d, generator=g)
    return x


def test_ivfpq_self_recall_and_roundtrip(tmp_path):
    x = _data()
    idx = IVFPQIndex(64, 32, 16, device="cpu")
    idx.train(x, niter=6)
    idx.add(x[:2500])
    idx.add(x[2500:])                    # incremental add keeps lists sorted
    assert idx.ntotal == 4000 and int(idx.list_off[-1]) == 4000
    q = x[:32] + 0.05 * torch.randn(32, 64)
    D, I = idx.search(q, 5, nprobe=8)
    assert (I[:, 0] == torch.arange(32)).float().mean() > 0.9
    assert torch.all(D[:, :-1] <= D[:, 1:])
    f = FlatIndex(64, "l2", "cpu")
    f.add(x)
    _, If = f.search(q, 10)
    recall = sum(int(I[i, 0]) in If[i].tolist() for i in range(32)) / 32
    assert recall > 0.9
    p = tmp_path / "a.ivfpq"
    idx.save(p)
    back = faiss_io.read_index(p)
    assert isinstance(back, IVFPQIndex) and back.ntotal == 4000 and back.M == 16
    D2, I2 = back.search(q, 5, nprobe=8)
    assert torch.equal(I, I2)


def test_ivfpq_custom_ids_and_empty_probe():
    x = _data(600, 32, 1)
    idx = IVFPQIndex(32, 8, 8, device="cpu")
    idx.train(x, niter=4)
    idx.add(x, ids=torch.arange(600) * 10 + 7)
    D, I = idx.search(x[:4], 3, nprobe=2)
    assert all(int(i) % 10 == 7 for i in I.flatten() if i >= 0)


def test_refine_flat_improves_recall_cpu():
    """Exact re-ranking of IVF-PQ candidates: recall@k rises to the candidates' coverage
    and refined distances are exact."""
    import torch

    from docqa_amd.index.ivfpq import IVFPQIndex
    from docqa_amd.index.refine import RefineFlat

    g = torch.Generator().manual_seed(0)
    d, n = 32, 3000
    xb = torch.randn(n, d, generator=g)
    xq = xb[:20] + 0.05 * torch.randn(20, d, generator=g)
    idx = IVFPQIndex(d, 16, 8, device="cpu")
    idx.train(xb, niter=5)
    idx.add(xb)
    exact = torch.cdist(xq, xb).topk(5, largest=False).indices
    _, Ia = idx.search(xq, 5, nprobe=16)
    ref = RefineFlat(idx, xb, k_factor=6)
    Dr, Ir = ref.search(xq, 5, nprobe=16)
    rec = lambda I: sum(len(set(I[i].tolist()) & set(exact[i].tolist())) for i in range(20)) / 100
    assert rec(Ir) >= rec(Ia) and rec(Ir) >= 0.8
    true_d = ((xb[Ir[:, 0]] - xq) ** 2).sum(-1)
    assert torch.allclose(Dr[:, 0], true_d, atol=1e-3)
