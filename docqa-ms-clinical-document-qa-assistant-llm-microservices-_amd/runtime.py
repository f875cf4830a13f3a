"""Handles to the native (C++) runtime objects compiled into ``ops/_docqa_C.so``.

* ``torch.classes.docqa_rt.BlockManager`` -- paged-KV block allocator with refcounts
  and a content-hashed prompt-prefix cache (csrc/runtime/block_manager.cpp).
"""
from __future__ import annotations

import torch

from . import ops

# the block manager's pool-exhaustion message (csrc/runtime/block_manager_core.h)
_EXHAUSTED = "KV cache exhausted"


class NativeBlockAllocator:
    """Python-facing wrapper with the :class:`engine.kv_cache.PyBlockAllocator` API."""

    def __init__(self, num_blocks: int, block_size: int = 64):
        self._m = torch.classes.docqa_rt.BlockManager(num_blocks, block_size)
        self.num_blocks = num_blocks
        self.block_size = block_size

    def num_free(self) -> int:
        return int(self._m.num_free())

    def alloc(self, n: int) -> list[int]:
        try:
            return list(self._m.alloc(n))
        except RuntimeError as e:
            if _EXHAUSTED in str(e):
                raise MemoryError(str(e)) from e
            raise

    def share(self, blocks: list[int]) -> None:
        self._m.share(list(blocks))

    def free(self, blocks: list[int]) -> None:
        self._m.free(list(blocks))

    def match_prefix(self, tokens: list[int]) -> list[int]:
        return list(self._m.match_prefix(list(tokens)))

    def register_prefix(self, tokens: list[int], blocks: list[int]) -> None:
        self._m.register_prefix(list(tokens), list(blocks))

    def match_alloc_batch(self, keys: list[list[int]], lens: list[int], need: list[int]):
        """One native call for a whole batch (block_manager_core.h match_alloc_batch):
        ``keys[i]``: chained keys of prompt i's full blocks.  Returns (hits, tables)."""
        flat = [k for ks in keys for k in ks]
        try:
            out = self._m.match_alloc_batch(flat, [len(ks) for ks in keys], list(lens), list(need))
        except RuntimeError as e:
            # only pool exhaustion is transient; invariant violations (bad sizes, ids out of
            # range, double free) must surface as the corruption they are
            if _EXHAUSTED in str(e):
                raise MemoryError(str(e)) from e
            raise
        B = len(keys)
        hits, tables, o = list(out[:B]), [], B
        for n in need:
            tables.append(list(out[o:o + n]))
            o += n
        return hits, tables

    def register_batch(self, keys: list[list[int]], tables: list[list[int]]) -> None:
        self._m.register_batch([k for ks in keys for k in ks], [len(ks) for ks in keys],
                               [b for tb in tables for b in tb], [len(tb) for tb in tables])

    def stats(self) -> dict:
        f, lru, cached, lookups, hits = self._m.stats()
        return {"free": f, "evictable": lru, "cached_blocks": cached, "lookups": lookups,
                "hit_blocks": hits}


def native_block_allocator(num_blocks: int, block_size: int = 64):
    if not ops.load_native():
        return None
    try:
        return NativeBlockAllocator(num_blocks, block_size)
    except Exception:
        return None
