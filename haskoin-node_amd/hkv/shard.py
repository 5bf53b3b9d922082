"""Signature-index sharding across GPUs: contiguous ranges,
64-aligned starts (a wave's ballot word pair never straddles two ranks), the
remainder on the last rank. The same rule as hkv_api.cpp's in-process
sharding, so a 1-GPU and an N-GPU run produce bit-identical bitmaps.

``ShardedVerify`` is one rank's step of the one-process-per-GPU run that
bench.py times: verify the rank's shard into its verdict words, then ONE
all-gather of every rank's words (RCCL over xGMI on the GPU box; the only
collective on the path), then ``bitmap()`` assembles the global bitmap."""
from __future__ import annotations

from typing import Callable, Tuple

import numpy as np


def shard_bounds(n: int, rank: int, world: int) -> Tuple[int, int]:
    per = -(-n // world) if world else n
    per = -(-per // 64) * 64
    lo = min(n, rank * per)
    hi = min(n, lo + per)
    if rank == world - 1:
        hi = n
    return lo, hi


def words_per_rank(n: int, world: int) -> int:
    """uint32 words in each rank's all-gather slot: the largest shard's
    ballot words (two per 64 signatures) plus two spare."""
    longest = max(hi - lo for lo, hi in (shard_bounds(n, r, world) for r in range(world)))
    return (longest + 63) // 64 * 2 + 2


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


class ShardedVerify:
    """One rank's verify step over its shard of an n-signature batch.

    verify: called as verify(lo, hi, bits) — must write the verdict words of
    records [lo, hi) into the int32 tensor ``bits`` (hkv_verify_device on the
    rank's GPU in bench.py; a CPU checker in the gloo tests).
    dist: torch.distributed (None, or world == 1 without force_collective:
    no collective).
    force_collective: keep the all-gather at world == 1 (bench.py
    --force-collective: a one-rank RCCL group, so the N > 1 step's device
    collective runs on a 1-GPU lease).
    gather_on_host: the all-gather runs on host copies of the words (a gloo
    group: bench.py --share-device, every rank on one GPU, which RCCL does
    not allow)."""

    def __init__(self, torch, n: int, rank: int, world: int, verify: Callable, dist=None, device: str = "cuda",
                 gather_on_host: bool = False, force_collective: bool = False):
        self.n, self.rank, self.world = n, rank, world
        self.lo, self.hi = shard_bounds(n, rank, world)
        self.wpr = words_per_rank(n, world)
        self.verify = verify
        self.dist = dist if (world > 1 or force_collective) else None
        self.bits = torch.zeros(self.wpr, dtype=torch.int32, device=device)
        gdev = "cpu" if gather_on_host else device
        self.host_bits = torch.zeros(self.wpr, dtype=torch.int32, device="cpu") \
            if gather_on_host and self.dist else None
        self.gathered = torch.zeros(self.wpr * world, dtype=torch.int32, device=gdev) if self.dist else None

    @property
    def local_n(self) -> int:
        return self.hi - self.lo

    def step(self) -> None:
        """Verify the shard, then the one all-gather of the verdict words."""
        self.verify(self.lo, self.hi, self.bits)
        if self.dist is not None:
            if self.host_bits is not None:
                self.host_bits.copy_(self.bits)  # (synchronous D2H: after the verify on the current stream)
                self.dist.all_gather_into_tensor(self.gathered, self.host_bits)
            else:
                self.dist.all_gather_into_tensor(self.gathered, self.bits)

    def local_bitmap(self) -> np.ndarray:
        """This rank's own verdict words for records [lo, hi) as verify()
        wrote them (before any collective): ceil((hi - lo) / 32) words."""
        return self.bits.cpu().numpy().view(np.uint32)[: (self.hi - self.lo + 31) // 32].copy()

    def bitmap(self) -> np.ndarray:
        """The global verdict bitmap (ceil(n/32) words) after step()."""
        if self.dist is None:
            return self.bits.cpu().numpy().view(np.uint32)[: (self.n + 31) // 32].copy()
        return assemble_bitmap(self.n, self.world, self.gathered.cpu().numpy().view(np.uint32), self.wpr)

    def slice_mismatches(self, full: np.ndarray, labels: np.ndarray) -> int:
        """Records [lo, hi) of the assembled global bitmap ``full`` against
        this rank's construction labels (uint32 words, bit 0 = record lo).
        Summed over ranks this checks every bit of the gathered bitmap."""
        n = self.hi - self.lo
        if n == 0:
            return 0
        got = np.unpackbits(full.view(np.uint8), bitorder="little")[self.lo:self.hi]
        want = np.unpackbits(np.ascontiguousarray(labels).view(np.uint8), bitorder="little")[:n]
        return int((got != want).sum())
