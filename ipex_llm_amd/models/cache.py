"""Paged KV cache sized for MI355X's 288 GB HBM.

Reference: ``SRC/transformers/kv.py`` (DynamicNormalCache / DynamicFp8Cache:
contiguous caches grown 256 tokens at a time, fp8 as uint8) and the vLLM
block tables of ``VLLM_PATCH`` (reshape_and_cache / paged attention).

Here every layer owns two tensors ``[num_blocks, Hkv, block_size, D]``
(bf16/fp16, or fp8 bytes).  A sequence owns a list of blocks (its row of the
int32 block table).  Static single-request generation simply reserves
``ceil(max_len / bs)`` blocks per sequence up front -- there is no regrowth
(and so no re-allocation inside a captured hipGraph).
"""
from __future__ import annotations

from typing import List, Optional

import torch

KV_FP8_NONE, KV_FP8_E5M2, KV_FP8_E4M3 = 0, 1, 2


class BlockAllocator:
    def __init__(self, num_blocks: int):
        self.free: List[int] = list(range(num_blocks - 1, -1, -1))

    def alloc(self, n: int) -> List[int]:
        if n > len(self.free):
            raise RuntimeError(f"KV cache exhausted: need {n} blocks, {len(self.free)} free")
        return [self.free.pop() for _ in range(n)]

    def release(self, blocks: List[int]):
        self.free.extend(reversed(blocks))


class PagedKVCache:
    def __init__(self, num_layers: int, num_blocks: int, num_kv_heads: int, head_dim: int,
                 block_size: int = 64, dtype=torch.bfloat16, device="cuda", kv_fp8: int = 0,
                 k_scale: float = 1.0, v_scale: float = 1.0):
        if block_size % 64:
            raise ValueError("block_size must be a multiple of 64")
        self.num_layers, self.num_blocks = num_layers, num_blocks
        self.Hkv, self.D, self.bs = num_kv_heads, head_dim, block_size
        self.dtype, self.kv_fp8 = dtype, kv_fp8
        self.k_scale, self.v_scale = k_scale, v_scale
        store = torch.uint8 if kv_fp8 else dtype
        shape = (num_blocks, num_kv_heads, block_size, head_dim)
        self.k = [torch.zeros(shape, dtype=store, device=device) for _ in range(num_layers)]
        self.v = [torch.zeros(shape, dtype=store, device=device) for _ in range(num_layers)]
        self.allocator = BlockAllocator(num_blocks)
        self.device = torch.device(device)

    @staticmethod
    def bytes_per_token(num_layers, num_kv_heads, head_dim, dtype=torch.bfloat16, kv_fp8=0):
        eb = 1 if kv_fp8 else torch.empty(0, dtype=dtype).element_size()
        return 2 * num_layers * num_kv_heads * head_dim * eb

    def blocks_for(self, n_tokens: int) -> int:
        return (n_tokens + self.bs - 1) // self.bs


class SequenceState:
    """Host-side bookkeeping of one sequence in the cache."""

    def __init__(self, blocks: List[int], length: int = 0):
        self.blocks = blocks
        self.length = length


def make_block_table(seqs: List[SequenceState], max_blocks: int, device) -> torch.Tensor:
    t = torch.zeros(len(seqs), max_blocks, dtype=torch.int32)
    for i, s in enumerate(seqs):
        t[i, :len(s.blocks)] = torch.tensor(s.blocks, dtype=torch.int32)
    return t.to(device)


def slots_for(seq: SequenceState, start: int, n: int, bs: int) -> torch.Tensor:
    pos = torch.arange(start, start + n)
    blk = torch.tensor(seq.blocks, dtype=torch.int64)[pos // bs]
    return blk * bs + pos % bs
