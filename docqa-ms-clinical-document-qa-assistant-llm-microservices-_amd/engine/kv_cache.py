"""Paged KV cache sized for 288 GB of HBM3E per MI355X.

Layout per layer: ``k_cache, v_cache : [num_blocks, Hkv_local, BS, D]`` bf16, so one
(block, kv-head) is ``BS*D*2`` contiguous bytes (16 KiB at BS=64, D=128) -- the
decode kernel streams it with 1 KiB wave instructions and the prefill scatter writes
whole 256-B rows.

Block bookkeeping is done by the native allocator in ``csrc/runtime/block_manager.cpp``
when the extension is loaded (O(1) alloc/free, refcounts for shared prompt prefixes)
and by the pure-Python :class:`PyBlockAllocator` otherwise.
"""
from __future__ import annotations

import torch


class PyBlockAllocator:
    """Free-list block allocator (reference implementation of the native one)."""

    def __init__(self, num_blocks: int):
        self.num_blocks = num_blocks
        self._free = list(range(num_blocks - 1, -1, -1))
        self._ref = [0] * num_blocks

    def num_free(self) -> int:
        return len(self._free)

    def alloc(self, n: int) -> list[int]:
        if n > len(self._free):
            raise MemoryError(f"KV cache exhausted: need {n} blocks, {len(self._free)} free")
        out = [self._free.pop() for _ in range(n)]
        for b in out:
            self._ref[b] = 1
        return out

    def share(self, blocks: list[int]) -> None:
        for b in blocks:
            self._ref[b] += 1

    def free(self, blocks: list[int]) -> None:
        for b in blocks:
            self._ref[b] -= 1
            if self._ref[b] == 0:
                self._free.append(b)
            elif self._ref[b] < 0:
                raise RuntimeError(f"double free of KV block {b}")


def make_allocator(num_blocks: int, block_size: int = 64):
    try:
        from ..runtime import native_block_allocator

        a = native_block_allocator(num_blocks, block_size)
        if a is not None:
            return a
    except Exception:
        pass
    return PyBlockAllocator(num_blocks)


class KVCache:
    def __init__(self, layers: int, num_blocks: int, kv_heads: int, head_dim: int,
                 block_size: int = 64, device="cuda", dtype=torch.bfloat16):
        if block_size & (block_size - 1):
            raise ValueError("block_size must be a power of two")
        self.block_size = block_size
        self.num_blocks = num_blocks
        shape = (num_blocks, kv_heads, block_size, head_dim)
        self.caches = [(torch.empty(shape, device=device, dtype=dtype),
                        torch.empty(shape, device=device, dtype=dtype)) for _ in range(layers)]
        self.allocator = make_allocator(num_blocks, block_size)

    @staticmethod
    def bytes_per_block(layers, kv_heads, head_dim, block_size, dtype_bytes=2) -> int:
        return 2 * layers * kv_heads * head_dim * block_size * dtype_bytes

    @classmethod
    def for_budget(cls, layers, kv_heads, head_dim, budget_bytes, block_size=64, device="cuda",
                   dtype=torch.bfloat16):
        nb = max(1, budget_bytes // cls.bytes_per_block(layers, kv_heads, head_dim, block_size))
        return cls(layers, int(nb), kv_heads, head_dim, block_size, device, dtype)

    def blocks_for(self, tokens: int) -> int:
        return (tokens + self.block_size - 1) // self.block_size
