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


class TailCache:
    """Token-granular extension of the block prefix cache (RadixAttention-style reuse below
    the 64-token block granularity).

    The block prefix cache shares a prompt's leading FULL blocks with an earlier prompt.
    Where two RAG prompts diverge inside a block -- at a retrieved-chunk boundary or in the
    question -- the tokens of that block before the divergence point are identical too,
    and so are their K/V (causal attention: position t depends only on tokens <= t).  This
    cache remembers, for every block position of every prefilled prompt, (block id, the
    prompt's tokens in that block), indexed by a chain hash of all tokens before the block
    and the block's first token.  A new prompt whose full-block match stops at block k
    looks block k up here; the longest common token run m over the stored variants is
    copied into the prompt's own fresh block (a K/V row copy instead of m tokens of
    prefill) and prefill starts at 64 k + m.

    Each entry pins its block (one allocator reference), so the rows it promises are never
    reallocated; entries are evicted least-recently-used beyond ``capacity``.  Thread-safe
    (the pipelined RAG prep thread reserves while the main thread registers)."""

    SEED = 0x243F6A88

    def __init__(self, allocator, block_size: int, capacity: int = 1024):
        import collections
        import threading

        self.alloc = allocator
        self.bs = block_size
        self.capacity = capacity
        # LRU over entries: (prefix key, block) -> tokens; index (prefix key, first token)
        # -> {block: tokens}
        self._lru: "collections.OrderedDict[tuple[int, int], tuple]" = collections.OrderedDict()
        self._idx: dict[tuple[int, int], dict[int, tuple]] = {}
        self._lock = threading.Lock()
        self.lookups = 0
        self.hit_tokens = 0

    def __len__(self) -> int:
        return len(self._lru)

    def _chain(self, tokens, nblocks: int) -> list[int]:
        """keys[j]: key of block position j = chain hash of every token before it."""
        bs, h = self.bs, self.SEED
        out = [h]
        for j in range(nblocks):
            h = hash((h, tuple(tokens[j * bs:(j + 1) * bs])))
            out.append(h)
        return out

    def _drop(self, key: int, blk: int) -> None:
        toks = self._lru.pop((key, blk))
        variants = self._idx.get((key, toks[0]))
        if variants is not None:
            variants.pop(blk, None)
            if not variants:
                del self._idx[(key, toks[0])]

    def lookup(self, tokens, k: int, limit: int) -> tuple[int, int] | None:
        """(source block, m): the longest cached token run at block position ``k`` that
        ``tokens`` continue, m <= ``limit``; pins the source block (release it with
        :meth:`unpin` once the copy is queued).  None when nothing matches."""
        if limit <= 0:
            return None
        key = self._chain(tokens, k)[k]
        seg = tokens[k * self.bs:k * self.bs + min(self.bs, limit)]
        with self._lock:
            self.lookups += 1
            variants = self._idx.get((key, seg[0]))
            if not variants:
                return None
            best, bm = -1, 0
            for blk, toks in variants.items():
                m, n = 1, min(len(toks), len(seg))
                while m < n and toks[m] == seg[m]:
                    m += 1
                if m > bm:
                    best, bm = blk, m
            self._lru.move_to_end((key, best))
            self.alloc.share([best])
            self.hit_tokens += bm
            return best, bm

    def unpin(self, blocks: list[int]) -> None:
        if blocks:
            self.alloc.free(blocks)

    def register(self, tokens, table: list[int]) -> None:
        """Publish every block position of a prefilled prompt (its prompt tokens only: the
        rows past the prompt belong to generation)."""
        bs = self.bs
        nb = min((len(tokens) + bs - 1) // bs, len(table))
        keys = self._chain(tokens, nb)
        freed = []
        with self._lock:
            for j in range(nb):
                toks = tuple(tokens[j * bs:(j + 1) * bs])
                key, blk = keys[j], table[j]
                if (key, blk) in self._lru:
                    self._lru.move_to_end((key, blk))
                    continue
                variants = self._idx.setdefault((key, toks[0]), {})
                covered = None
                for b2, t2 in variants.items():
                    if t2[:len(toks)] == toks:   # an entry already promises these tokens
                        covered = b2
                        break
                if covered is not None:
                    self._lru.move_to_end((key, covered))
                    continue
                self.alloc.share([blk])
                variants[blk] = toks
                self._lru[(key, blk)] = toks
            while len(self._lru) > self.capacity:
                (key, blk), _ = next(iter(self._lru.items()))
                self._drop(key, blk)
                freed.append(blk)
        if freed:
            self.alloc.free(freed)

    def shrink(self, n: int) -> int:
        """Evict the ``n`` least-recently-used entries (allocation pressure)."""
        freed = []
        with self._lock:
            for _ in range(min(n, len(self._lru))):
                (key, blk), _ = next(iter(self._lru.items()))
                self._drop(key, blk)
                freed.append(blk)
        if freed:
            self.alloc.free(freed)
        return len(freed)

    def clear(self) -> None:
        self.shrink(len(self._lru))
