"""IVF-PQ as the semantic-indexer's store (INDEX_TYPE=ivfpq, index/hybrid.py): exact flat
search until trained, IVF-PQ + exact refine after, FAISS IndexRefineFlat (IxRF) snapshots
that resume into a trained store, the index follower of a multi-process deployment, and
a sharded IVF-PQ (shared quantizers, per-rank lists, all-gather merge) equal to one IVF-PQ
over all vectors."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from docqa_amd.index import faiss_io
from docqa_amd.index.flat import FlatIndex
from docqa_amd.index.hybrid import IVFPQRefineIndex


def _data(n=3000, d=32, nq=20, seed=0):
    g = torch.Generator().manual_seed(seed)
    lat = torch.randn(n, 8, generator=g)
    A = torch.randn(8, d, generator=g)
    xb = lat @ A + 0.05 * torch.randn(n, d, generator=g)
    xq = xb[torch.randint(0, n, (nq,), generator=g)] + 0.05 * torch.randn(nq, d, generator=g)
    return xb, xq


def test_exact_until_trained_then_refined_recall(tmp_path):
    xb, xq = _data()
    idx = IVFPQRefineIndex(32, nlist=16, M=8, nprobe=8, k_factor=4, train_min=1000, device="cpu")
    flat = FlatIndex(32, "l2", device="cpu")
    idx.add(xb[:500])
    flat.add(xb[:500])
    assert not idx.trained
    assert torch.equal(idx.search(xq, 5)[1], flat.search(xq, 5)[1])      # exact before training
    idx.add(xb[500:])
    flat.add(xb[500:])
    assert idx.trained and idx.ntotal == 3000 and idx.ivf.ntotal == 3000
    _, I = idx.search(xq, 10)
    _, E = flat.search(xq, 10)
    recall = sum(len(set(a.tolist()) & set(b.tolist())) for a, b in zip(I, E)) / E.numel()
    assert recall >= 0.8, recall
    # IxRF snapshot -> resumes trained, same answers
    p = tmp_path / "vector_store.faiss"
    idx.save(p)
    assert p.read_bytes()[:4] == b"IxRF"
    data = faiss_io.read_index(p)
    assert isinstance(data, faiss_io.RefineIndexData) and data.ntotal == 3000
    again = IVFPQRefineIndex.load(p, device="cpu")
    assert again.trained and torch.equal(again.search(xq, 10)[1], I)


def test_indexer_service_with_ivfpq_store(tmp_path, monkeypatch):
    from docqa_amd.config import Settings
    from docqa_amd.index.follower import IndexFollower
    from docqa_amd.models.bert import BertConfig, BertEncoder
    from docqa_amd.services.indexer import SemanticIndexer
    from docqa_amd.text.tokenizer import WordPieceTokenizer

    for k, v in {"INDEX_TYPE": "ivfpq", "IVF_NLIST": "8", "IVF_TRAIN_MIN": "400", "PQ_M": "8",
                 "IVF_NPROBE": "8", "INDEX_SNAPSHOT_EVERY": "1"}.items():
        monkeypatch.setenv(k, v)
    st = Settings()
    st.index_dir = str(tmp_path)
    enc = BertEncoder(BertConfig.preset("tiny-bert"), device="cpu")
    idx = SemanticIndexer(enc, WordPieceTokenizer(), st, device="cpu").startup()   # KB bootstrap (649 rows)
    assert isinstance(idx.index, IVFPQRefineIndex) and idx.index.trained
    n0 = idx.index.ntotal
    idx.index_document(7, "Patient sous warfarine, INR instable. " * 30, {"patient_id": "P7"})
    idx.commit()
    assert idx.index.ntotal > n0 and idx.index.ivf.ntotal == idx.index.ntotal
    hits = idx.search("warfarine INR", k=3)
    assert len(hits) == 3
    # resume from the IxRF snapshot (+ WAL) and follow it from another "process"
    again = SemanticIndexer(enc, WordPieceTokenizer(), st, device="cpu").startup()
    assert isinstance(again.index, IVFPQRefineIndex) and again.index.trained
    assert again.index.ntotal == idx.index.ntotal
    fol = IndexFollower(st.index_dir, st.index_file, st.metadata_file, d=enc.cfg.hidden, device="cpu", settings=st)
    fol.poll()
    assert fol.index.ntotal == idx.index.ntotal and fol.index.trained
    q = enc.encode(WordPieceTokenizer().encode_batch(["warfarine INR"]))
    assert torch.equal(fol.index.search(q, 3)[1], idx.index.search(q, 3)[1])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_worker(rank, world, port, path, out, rotation="none"):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    from docqa_amd.index.ivfpq import IVFPQIndex
    from docqa_amd.index.sharded import ShardedIVFPQIndex
    from docqa_amd.parallel import comm

    comm.init_distributed(tp_size=1, backend="gloo")
    d = torch.load(path, weights_only=True)
    xb, xq = d["xb"], d["xq"]
    n = xb.shape[0]
    lo, hi = n * rank // world, n * (rank + 1) // world
    sh = ShardedIVFPQIndex.build(xb[lo:hi], d=xb.shape[1], nlist=16, M=8, train_sample=xb[:2000] if rank == 0 else None,
                                 device="cpu", rotation=rotation)
    D, I = sh.search(xq[rank::world], 10, nprobe=8)
    torch.save({"D": D, "I": I}, f"{out}.{rank}")
    comm.destroy()


@pytest.mark.parametrize("rotation", ["none", "pca"])
def test_sharded_ivfpq_equals_single(tmp_path, rotation):
    """Rank 0 trains the quantizers (and the PCA pre-rotation) and broadcasts them: every
    shard encodes alike, so the merged search equals one index over all vectors."""
    from docqa_amd.index.ivfpq import IVFPQIndex

    xb, xq = _data(n=4000, nq=12, seed=3)
    single = IVFPQIndex(32, 16, 8, device="cpu", rotation=rotation)
    single.train(xb[:2000])
    single.add(xb)
    path, out = tmp_path / "d.pt", tmp_path / "o"
    torch.save({"xb": xb, "xq": xq}, path)
    mp.start_processes(_shard_worker, args=(2, _free_port(), str(path), str(out), rotation), nprocs=2,
                       join=True, start_method="spawn")
    for r in range(2):
        got = torch.load(f"{out}.{r}", weights_only=True)
        D, I = single.search(xq[r::2], 10, nprobe=8)
        torch.testing.assert_close(got["D"], D, rtol=1e-4, atol=1e-4)
        # equal distances may come back in either order: compare id sets per distance
        assert torch.equal(torch.sort(got["I"], 1).values, torch.sort(I, 1).values)
