"""Paged KV cache (HBM) and its host-side block allocator.

Layout (one tensor per K and V for all layers, so a layer's cache is a contiguous view):

* K: [L, blocks, Hkv_local, 32, 128] bf16 — one key row = 256 contiguous bytes
* V: [L, blocks, Hkv_local, 128, 32] bf16 — transposed pages, tokens permuted by ``vperm``

Pages are 32 tokens.  At TP=1 Mistral-7B needs 128 KiB per token, so 100 GB of the 288 GB HBM holds
~780k tokens (about 190 sequences of 4k context per GPU).  The cache is zero-initialised so keys
past a sequence's end inside its last page are finite (they are masked, but 0·NaN would poison PV).
"""
from __future__ import annotations

import torch

PAGE = 32


class KVCache:
    def __init__(self, num_layers: int, num_blocks: int, nkv: int, device, dtype=torch.bfloat16):
        self.num_layers, self.num_blocks, self.nkv = num_layers, num_blocks, nkv
        self.k = torch.zeros(num_layers, num_blocks, nkv, PAGE, 128, device=device, dtype=dtype)
        self.v = torch.zeros(num_layers, num_blocks, nkv, 128, PAGE, device=device, dtype=dtype)

    @staticmethod
    def bytes_per_block(num_layers: int, nkv: int) -> int:
        return 2 * num_layers * nkv * PAGE * 128 * 2

    @classmethod
    def blocks_for_budget(cls, budget_bytes: int, num_layers: int, nkv: int) -> int:
        return max(1, budget_bytes // cls.bytes_per_block(num_layers, nkv))


class BlockAllocator:
    """Free-list allocator of KV pages (host side; the device only sees block tables)."""

    def __init__(self, num_blocks: int):
        self.num_blocks = num_blocks
        self._free = list(range(num_blocks - 1, -1, -1))

    @property
    def num_free(self) -> int:
        return len(self._free)

    def can_allocate(self, n: int) -> bool:
        return n <= len(self._free)

    def allocate(self, n: int) -> list:
        if n > len(self._free):
            raise MemoryError(f"KV cache exhausted: need {n} blocks, {len(self._free)} free")
        out = [self._free.pop() for _ in range(n)]
        return out

    def free(self, blocks) -> None:
        self._free.extend(reversed(list(blocks)))


def blocks_needed(num_tokens: int) -> int:
    return (num_tokens + PAGE - 1) // PAGE
