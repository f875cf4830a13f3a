"""On-disk compatibility with the reference's shipped index files (byte-exact)."""
import numpy as np
import pytest

from docqa_amd.index import faiss_io
from docqa_amd.store import metadata_io
from tests.helpers import REFERENCE_FAISS, REFERENCE_META

needs_ref = pytest.mark.skipif(not REFERENCE_FAISS.exists(), reason="reference not mounted")


@needs_ref
def test_read_shipped_faiss_header_and_norms():
    idx = faiss_io.read_index(REFERENCE_FAISS)
    assert idx.d == 384 and idx.ntotal == 649 and idx.metric == faiss_io.METRIC_L2
    norms = np.linalg.norm(idx.xb, axis=1)
    assert norms.min() > 0.9999 and norms.max() < 1.0001


@needs_ref
def test_roundtrip_byte_exact(tmp_path):
    raw = REFERENCE_FAISS.read_bytes()
    idx = faiss_io.read_index(REFERENCE_FAISS)
    out = tmp_path / "v.faiss"
    faiss_io.write_flat(out, idx.xb, idx.metric)
    assert out.read_bytes() == raw


@needs_ref
def test_read_shipped_metadata_restricted():
    rows = metadata_io.read_metadata(REFERENCE_META)
    assert len(rows) == 649
    assert all(set(metadata_io.REQUIRED_KEYS) <= set(r) for r in rows)
    assert rows[647]["source"] == "Dossier Patient 1"
    assert rows[0]["type"] == "knowledge_base"


@needs_ref
def test_metadata_roundtrip_byte_exact(tmp_path):
    rows = metadata_io.read_metadata(REFERENCE_META)
    p = tmp_path / "m.pkl"
    metadata_io.write_metadata(p, rows)
    assert metadata_io.read_metadata(p) == rows


def test_restricted_unpickler_refuses_globals():
    import pickle

    class Evil:
        def __reduce__(self):
            return (print, ("pwned",))

    with pytest.raises(pickle.UnpicklingError):
        metadata_io.loads_metadata(pickle.dumps([Evil()]))


def test_flat_ip_roundtrip(tmp_path):
    xb = np.random.RandomState(0).randn(10, 16).astype(np.float32)
    p = tmp_path / "ip.faiss"
    faiss_io.write_flat(p, xb, faiss_io.METRIC_INNER_PRODUCT)
    back = faiss_io.read_index(p)
    assert back.metric == faiss_io.METRIC_INNER_PRODUCT
    np.testing.assert_array_equal(back.xb, xb)


def test_truncated_file_rejected(tmp_path):
    p = tmp_path / "bad.faiss"
    p.write_bytes(faiss_io.flat_bytes(np.ones((4, 8), np.float32))[:-10])
    with pytest.raises(ValueError):
        faiss_io.read_index(p)


def test_segment_log_replay_and_torn_tail(tmp_path):
    """WAL frames replay in order after a snapshot's sequence number; a torn tail (crash
    mid-append) is dropped and truncated; reset starts an empty log."""
    import numpy as np

    from docqa_amd.store.segment_log import SegmentLog

    p = tmp_path / "idx.wal"
    log = SegmentLog(p, fsync=False)
    v = np.arange(12, dtype=np.float32).reshape(3, 4)
    log.append([{"a": 1}, {"a": 2}, {"a": 3}], v)
    log.append([{"b": 1}], v[:1] * 2)
    log.close()
    with open(p, "ab") as f:          # torn third frame
        f.write(b"DQW1" + b"\x00" * 10)
    size_torn = p.stat().st_size
    got = list(SegmentLog(p).replay())
    assert [s for s, _, _ in got] == [1, 2] and got[0][1][2] == {"a": 3}
    assert np.array_equal(got[1][2], v[:1] * 2)
    assert p.stat().st_size < size_torn
    assert [s for s, _, _ in SegmentLog(p).replay(after_seq=1)] == [2]
    log2 = SegmentLog(p, fsync=False)
    list(log2.replay())
    log2.reset(2)
    assert p.stat().st_size == 0 and log2.append([{"c": 1}], v[:1]) == 3


def test_indexer_wal_resume_without_snapshot(tmp_path):
    """Batches acked on a WAL append survive a restart that never saw a snapshot: the new
    indexer loads the last snapshot and replays the log (same vectors, same metadata)."""
    import torch

    from docqa_amd.config import Settings
    from docqa_amd.models.bert import BertConfig, BertEncoder
    from docqa_amd.services.indexer import SemanticIndexer
    from docqa_amd.text.tokenizer import WordPieceTokenizer

    st = Settings()
    st.index_dir = str(tmp_path)
    st.default_data_dir = str(tmp_path / "nodata")
    st.snapshot_every = 1000
    enc = BertEncoder(BertConfig.preset("tiny-bert"), device="cpu")
    tok = WordPieceTokenizer()
    a = SemanticIndexer(enc, tok, st, device="cpu").startup(build_if_missing=True)
    n0 = a.index.ntotal
    for d in range(3):
        a.index_document(100 + d, f"Patient {d}: syndrome Vide de Qi. " * 30)
        a.commit()
    assert a._batches_since_snapshot == 3          # no snapshot taken since startup
    b = SemanticIndexer(enc, tok, st, device="cpu").startup(build_if_missing=True)
    assert b.index.ntotal == a.index.ntotal > n0
    assert [m["doc_id"] for m in b.metadata] == [m["doc_id"] for m in a.metadata]
    assert torch.allclose(b.index.xb.float(), a.index.xb.float())
    c = SemanticIndexer(enc, tok, st, device="cpu").startup()   # b snapshotted: nothing to replay
    assert c.index.ntotal == a.index.ntotal and c.wal.bytes == 0


def test_index_follower_tails_writer_across_snapshots(tmp_path):
    """A reader process's follower sees every batch the indexer makes durable (WAL tail),
    keeps them across the writer's snapshot rotations, and reloads the snapshot when it
    missed frames."""
    import torch

    from docqa_amd.config import Settings
    from docqa_amd.index.follower import IndexFollower
    from docqa_amd.models.bert import BertConfig, BertEncoder
    from docqa_amd.services.indexer import SemanticIndexer
    from docqa_amd.text.tokenizer import WordPieceTokenizer

    st = Settings()
    st.index_dir = str(tmp_path)
    st.default_data_dir = str(tmp_path / "nodata")
    st.snapshot_every = 2
    enc = BertEncoder(BertConfig.preset("tiny-bert"), device="cpu")
    w = SemanticIndexer(enc, WordPieceTokenizer(), st, device="cpu").startup(build_if_missing=True)
    f = IndexFollower(str(tmp_path), d=enc.cfg.hidden, device="cpu")
    f.poll()
    assert f.index.ntotal == w.index.ntotal == len(f.metadata)
    for d in range(5):                      # snapshots rotate the log every 2 batches
        w.index_document(200 + d, f"Note {d}: Vide de Qi, Rate. " * 25)
        w.commit()
        f.poll()
        assert f.index.ntotal == w.index.ntotal and len(f.metadata) == f.index.ntotal
    assert [m["doc_id"] for m in f.metadata] == [m["doc_id"] for m in w.metadata]
    assert torch.allclose(f.index.xb.float(), w.index.xb.float())
    g = IndexFollower(str(tmp_path), d=enc.cfg.hidden, device="cpu")   # late joiner
    w.index_document(300, "Late note. " * 40)
    w.commit()
    w.index_document(301, "Later note. " * 40)
    w.commit()                               # rotation happened before g ever polled
    g.poll()
    assert g.index.ntotal == w.index.ntotal


def test_index_follower_reload_is_atomic_for_concurrent_search(tmp_path):
    """Snapshot reloads swap vectors + metadata together: a search racing the reload never
    sees an empty / partial index or an id without its record."""
    import threading

    import torch

    from docqa_amd.config import Settings
    from docqa_amd.index.follower import IndexFollower
    from docqa_amd.models.bert import BertConfig, BertEncoder
    from docqa_amd.services.indexer import SemanticIndexer
    from docqa_amd.text.tokenizer import WordPieceTokenizer

    st = Settings()
    st.index_dir = str(tmp_path)
    st.default_data_dir = str(tmp_path / "nodata")
    enc = BertEncoder(BertConfig.preset("tiny-bert"), device="cpu")
    w = SemanticIndexer(enc, WordPieceTokenizer(), st, device="cpu").startup(build_if_missing=True)
    f = IndexFollower(str(tmp_path), d=enc.cfg.hidden, device="cpu")
    f.poll()
    n0 = f.index.ntotal
    assert n0 > 0
    q = torch.randn(4, enc.cfg.hidden)
    bad, stop = [], threading.Event()

    def searcher():
        while not stop.is_set():
            n = f.index.ntotal
            D, I = f.index.search(q, 3)
            if n < n0 or (I < 0).any() or int(I.max()) >= len(f.metadata):
                bad.append((n, I.tolist(), len(f.metadata)))

    t = threading.Thread(target=searcher)
    t.start()
    try:
        for _ in range(30):
            f._load_snapshot()
    finally:
        stop.set()
        t.join()
    assert not bad, bad[:3]
    assert f.index.ntotal == n0 == len(f.metadata)
