"""``metadata_store.pkl`` compatibility (semantic-indexer/indexer.py:26-30,43-48;
read back at llm-qa/main.py:37-38).

The reference stores a plain ``list[dict]`` (pickle protocol 4, builtin types only), one
dict per index row: ``doc_id``, ``text_content``, ``source``, ``type``.  We read it with
a *restricted* unpickler that refuses every GLOBAL/REDUCE (no code from the file is ever
executed) and write it with protocol 4 so the reference's llm-qa can still load our
files.  Writes are atomic.
"""
from __future__ import annotations

import io
import pickle
from pathlib import Path

from ..index.faiss_io import atomic_write

REQUIRED_KEYS = ("doc_id", "text_content", "source", "type")


class _SafeUnpickler(pickle.Unpickler):
    def find_class(self, module, name):  # noqa: D401 - pickle API
        raise pickle.UnpicklingError(f"refusing to load global {module}.{name} from metadata")


def loads_metadata(data: bytes) -> list[dict]:
    obj = _SafeUnpickler(io.BytesIO(data)).load()
    if not isinstance(obj, list) or not all(isinstance(r, dict) for r in obj):
        raise ValueError("metadata store must be a list of dicts")
    return obj


def read_metadata(path) -> list[dict]:
    return loads_metadata(Path(path).read_bytes())


def dumps_metadata(rows: list[dict]) -> bytes:
    clean = []
    for r in rows:
        clean.append({k: (v if isinstance(v, (str, int, float, bool, type(None))) else str(v))
                      for k, v in r.items()})
    return pickle.dumps(clean, protocol=4)


def write_metadata(path, rows: list[dict]) -> None:
    atomic_write(path, dumps_metadata(rows))
