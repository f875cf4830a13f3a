from pathlib import Path

REFERENCE = Path("/root/reference")
REFERENCE_FAISS = REFERENCE / "semantic-indexer" / "vector_store.faiss"
REFERENCE_META = REFERENCE / "semantic-indexer" / "metadata_store.pkl"
REFERENCE_CSV_DIR = REFERENCE / "semantic-indexer" / "default_data"
