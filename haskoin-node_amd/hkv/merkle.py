"""Batch block merkle roots — host-side mirror of haskoin-core
``buildMerkleRoot :: [TxHash] -> Hash256`` [dep, haskoin-core-1.1.0
Haskoin.Block.Merkle], which the reference checks against every fetched
block's header (/root/reference/test/Haskoin/NodeSpec.hs:185-193, blocks from
``getBlocks``, src/Haskoin/Node/Peer.hs:309-344). All hashing runs in libhkv's
HIP kernels (csrc/hkv_headers.hip), on one of two routes: batches of at most
n_cu blocks (256 on an MI355X) split each tree over 8 aligned-subtree
workgroups (hkv_merkle_sub_kernel) joined by hkv_merkle_top_kernel; larger
batches take one workgroup per block (hkv_merkle_kernel).

    merkle_roots(v, blocks) -> (roots: list of 32-byte digests, mutated: bool[n])

``blocks`` is a list of txid lists (32-byte txHash values in digest order).
``mutated`` is the CVE-2012-2459 duplicate-pair flag.
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence, Tuple

import numpy as np

from .lib import check


def merkle_roots(v, blocks: Sequence[Sequence[bytes]]) -> Tuple[List[bytes], np.ndarray]:
    """Batch buildMerkleRoot on the context's first device (blocking)."""
    nb = len(blocks)
    offsets = np.zeros(nb + 1, dtype=np.uint32)
    parts = []
    for b, txids in enumerate(blocks):
        for t in txids:
            if len(t) != 32:
                raise ValueError("a txid is 32 bytes")
        parts.extend(txids)
        offsets[b + 1] = offsets[b] + len(txids)
    leaves = np.frombuffer(b"".join(parts), dtype=np.uint8).copy() if parts else np.zeros(1, dtype=np.uint8)
    roots = np.zeros(nb * 32 + 1, dtype=np.uint8)
    mutated = np.zeros(nb + 1, dtype=np.uint8)
    rc = v.lib.hkv_merkle_roots(v.ctx, leaves.ctypes.data, offsets.ctypes.data, nb, roots.ctypes.data,
                                mutated.ctypes.data)
    check(rc, "hkv_merkle_roots", v.lib)
    rb = roots.tobytes()
    return [rb[32 * i: 32 * i + 32] for i in range(nb)], mutated[:nb].astype(bool)


def merkle_roots_device(v, dev: int, d_txids: int, d_offsets: int, n_blocks: int, d_scratch: int, d_roots: int,
                        d_mutated: int, stream: int = 0) -> None:
    """Device-pointer form (HBM-resident txid batches; enqueued, not synchronised)."""
    rc = v.lib.hkv_merkle_roots_device(v.ctx, dev, ctypes.c_void_p(d_txids), ctypes.c_void_p(d_offsets), n_blocks,
                                       ctypes.c_void_p(d_scratch), ctypes.c_void_p(d_roots),
                                       ctypes.c_void_p(d_mutated), ctypes.c_void_p(stream) if stream else None)
    check(rc, "hkv_merkle_roots_device", v.lib)
