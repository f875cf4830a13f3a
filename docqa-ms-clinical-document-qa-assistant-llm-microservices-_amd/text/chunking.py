"""Text chunking.

* :func:`chunk_chars` -- the reference's fixed-size character chunks
  (``[text[i:i+500] for i in range(0, len(text), 500)]``, semantic-indexer/indexer.py:120).
* :func:`chunk_tokens` -- token-budgeted chunks with overlap, cut on whitespace, so a
  chunk never exceeds the encoder's 256-token window (MiniLM truncates silently).
"""
from __future__ import annotations


def chunk_chars(text: str, size: int = 500) -> list[str]:
    if not text:
        return []
    return [text[i:i + size] for i in range(0, len(text), size)]


def chunk_tokens(text: str, count_tokens, max_tokens: int = 240, overlap_words: int = 16) -> list[str]:
    words = text.split()
    chunks, cur = [], []
    for w in words:
        cur.append(w)
        if count_tokens(" ".join(cur)) > max_tokens and len(cur) > 1:
            cur.pop()
            chunks.append(" ".join(cur))
            cur = cur[-overlap_words:] + [w] if overlap_words else [w]
    if cur:
        chunks.append(" ".join(cur))
    return chunks
