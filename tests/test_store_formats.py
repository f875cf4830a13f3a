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
