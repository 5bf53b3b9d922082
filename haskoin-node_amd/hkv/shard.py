"""Signature-index sharding across GPUs: contiguous ranges,
64-aligned starts (a wave's ballot word pair never straddles two ranks), the
remainder on the last rank. The same rule as hkv_api.cpp's in-process
sharding, so a 1-GPU and an N-GPU run produce bit-identical bitmaps."""
from __future__ import annotations

from typing import Tuple

import numpy as np


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    per = -(-n // world) if world else n
    per = -(-per // 64) * 64
    lo = min(n, rank * per)
    hi = min(n, lo + per)
    if rank == world - 1:
        hi = n
    return lo, hi


def assemble_bitmap(n: int, world: int, gathered_words: np.ndarray, words_per_rank: int) -> np.ndarray:
    """gathered_words: [world * words_per_rank] uint32 from an all-gather of
    each rank's shard bitmap (rank r's bits start at bit 0 of its slot).
    Returns the global bitmap of ceil(n/32) words."""
    out = np.zeros((n + 31) // 32, dtype=np.uint32)
    for r in range(world):
        lo, hi = shard_bounds(n, r, world)
        if hi <= lo:
            continue
        w = (hi - lo + 31) // 32
        out[lo // 32: lo // 32 + w] |= gathered_words[r * words_per_rank: r * words_per_rank + w]
    return out
