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
        # zeroed, not empty: the decode kernels stream whole 32-token tiles and mask the
        # positions past a sequence's end with p = 0, but 0 x NaN is NaN -- a never-written
        # slot holding a NaN bit pattern (whatever an earlier tensor of the process left
        # there) would poison the row.  Stale finite K/V of a reused block is harmless.
        self.caches = [(torch.zeros(shape, device=device, dtype=dtype),
                        torch.zeros(shape, device=device, dtype=dtype)) for _ in range(layers)]
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


def chain_keys(tokens, block_size: int, nblocks: int) -> list[int]:
    """keys[j] (j = 0 .. nblocks): chain hash of tokens [0, j * block_size) -- the key of
    block position j for the token-granular cache, and (j >= 1) of full block j - 1 for
    the block prefix cache (LLMEngine.reserve)."""
    h = TailCache.SEED
    out = [h]
    for j in range(nblocks):
        h = hash((h, tuple(tokens[j * block_size:(j + 1) * block_size])))
        out.append(h)
    return out


class TailCache:
    """Token-granular extension of the block prefix cache (RadixAttention-style reuse below
    the 64-token block granularity).

    The block prefix cache shares a prompt's leading FULL blocks with an earlier prompt.
    Where two RAG prompts diverge inside a block -- at a retrieved-chunk boundary or in the
    question -- the tokens of that block before the divergence point are identical too,
    and so are their K/V (causal attention: position t depends only on tokens <= t).  This
    cache remembers, for every block position of every prefilled prompt, (the prompt's
    tokens in that block, block id), keyed by a chain hash of all tokens before the block;
    the variants of one key are kept sorted, so the variant sharing the longest token run
    with a new prompt is a neighbour of its bisection point.  A prompt whose full-block
    match stops at block k copies the common K/V rows of that variant into its own fresh
    block (one gather/scatter per layer) and prefill starts at 64 k + m.

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
        # LRU over entries (prefix key, block) -> tokens; per key a sorted [(tokens, block)]
        self._lru: "collections.OrderedDict[tuple[int, int], tuple]" = collections.OrderedDict()
        self._var: dict[int, list[tuple[tuple, int]]] = {}
        self._lock = threading.Lock()
        self.lookups = 0
        self.hit_tokens = 0

    def __len__(self) -> int:
        return len(self._lru)

    def chain(self, tokens, nblocks: int) -> list[int]:
        """keys[j]: key of block position j = chain hash of every token before it."""
        return chain_keys(tokens, self.bs, nblocks)

    def _drop(self, key: int, blk: int) -> None:
        import bisect

        toks = self._lru.pop((key, blk))
        lst = self._var.get(key)
        if lst is not None:
            i = bisect.bisect_left(lst, (toks, blk))
            if i < len(lst) and lst[i] == (toks, blk):
                del lst[i]
            if not lst:
                del self._var[key]

    @staticmethod
    def _lcp(a: tuple, b) -> int:
        n, m = min(len(a), len(b)), 0
        while m < n and a[m] == b[m]:
            m += 1
        return m

    def lookup(self, tokens, k: int, limit: int, keys: list[int] | None = None) -> tuple[int, int] | None:
        """(source block, m): the longest cached token run at block position ``k`` that
        ``tokens`` continue, m <= ``limit``; pins the source block (release it with
        :meth:`unpin` once the copy is queued).  None when nothing matches.  ``keys``:
        precomputed :meth:`chain` of at least k blocks."""
        import bisect

        if limit <= 0:
            return None
        key = (keys if keys is not None else self.chain(tokens, k))[k]
        seg = tuple(tokens[k * self.bs:k * self.bs + min(self.bs, limit)])
        with self._lock:
            self.lookups += 1
            lst = self._var.get(key)
            if not lst:
                return None
            i = bisect.bisect_left(lst, (seg,))
            best, bm = -1, 0
            for j in (i - 1, i):
                if 0 <= j < len(lst):
                    m = self._lcp(lst[j][0], seg)
                    if m > bm:
                        best, bm = lst[j][1], m
            if bm == 0:
                return None
            self._lru.move_to_end((key, best))
            self.alloc.share([best])
            self.hit_tokens += bm
            return best, bm

    def unpin(self, blocks: list[int]) -> None:
        if blocks:
            self.alloc.free(blocks)

    def register(self, tokens, table: list[int], keys: list[int] | None = None) -> None:
        """Publish every block position of a prefilled prompt (its prompt tokens only: the
        rows past the prompt belong to generation)."""
        import bisect

        bs = self.bs
        nb = min((len(tokens) + bs - 1) // bs, len(table))
        if keys is None or len(keys) < nb + 1:
            keys = self.chain(tokens, nb)
        freed = []
        with self._lock:
            for j in range(nb):
                toks = tuple(tokens[j * bs:(j + 1) * bs])
                key, blk = keys[j], table[j]
                if (key, blk) in self._lru:
                    self._lru.move_to_end((key, blk))
                    continue
                lst = self._var.setdefault(key, [])
                i = bisect.bisect_left(lst, (toks,))
                if i < len(lst) and lst[i][0][:len(toks)] == toks:   # already promised
                    self._lru.move_to_end((key, lst[i][1]))
                    continue
                self.alloc.share([blk])
                lst.insert(i, (toks, blk))
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
