"""Batch block-header checks — the host-side mirror of the per-header work of
haskoin-node's header sync. All computation runs in
libhkv's HIP kernels (csrc/hkv_headers.hip).

Reference: ``importHeaders`` (/root/reference/src/Haskoin/Node/Chain.hs:500-520)
hands up to 2,000 headers per peer message to haskoin-core ``connectBlocks``
[dep, haskoin-core-1.1.0, /root/reference/stack.yaml:10], which needs per
header:

    headerHash :: BlockHeader -> BlockHash              -- SHA-256d, 80 bytes
    isValidPOW :: Network -> BlockHeader -> Bool        -- decodeCompact bits
    prev h == headerHash (previous header)              -- batch linkage

Batch equivalent (same per-element result):

    check_headers(v, headers, pow_limit, prev_hash=None)
        -> (hashes: list of 32-byte digests, status: uint8[n] of HKV_HDR_* flags)

The chain-context checks of connectBlocks (median time past, future-time
limit, nextWorkRequired, checkpoints, BIP34 height) stay on the host.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .lib import (HKV_HDR_ABOVE_LIMIT, HKV_HDR_HASH_ABOVE, HKV_HDR_LINK_OK, HKV_HDR_NEGATIVE,  # noqa: F401
                  HKV_HDR_OVERFLOW, HKV_HDR_POW_OK, HKV_HDR_ZERO_TARGET, check)

HEADER_SIZE = 80


def _limit_bytes(pow_limit: int) -> bytes:
    return int(pow_limit).to_bytes(32, "little")


def check_headers(v, headers: Sequence[bytes] | bytes | np.ndarray, pow_limit: int,
                  prev_hash: Optional[bytes] = None) -> Tuple[List[bytes], np.ndarray]:
    """Batch headerHash + isValidPOW + linkage on the context's first device."""
    if isinstance(headers, (bytes, bytearray, np.ndarray)):
        raw = np.frombuffer(bytes(headers), dtype=np.uint8) if not isinstance(headers, np.ndarray) else \
            np.ascontiguousarray(headers, dtype=np.uint8).reshape(-1)
    else:
        for h in headers:
            if len(h) != HEADER_SIZE:
                raise ValueError("a block header is 80 bytes")
        raw = np.frombuffer(b"".join(headers), dtype=np.uint8)
    if raw.size % HEADER_SIZE:
        raise ValueError("header batch is not a multiple of 80 bytes")
    n = raw.size // HEADER_SIZE
    if prev_hash is not None and len(prev_hash) != 32:
        raise ValueError("prev_hash is 32 bytes")
    hashes = np.zeros(n * 32, dtype=np.uint8)
    status = np.zeros(n, dtype=np.uint8)
    lim = np.frombuffer(_limit_bytes(pow_limit), dtype=np.uint8).copy()
    prev = None if prev_hash is None else np.frombuffer(prev_hash, dtype=np.uint8).copy()
    rc = v.lib.hkv_check_headers(v.ctx, raw.ctypes.data, n, lim.ctypes.data,
                                 None if prev is None else prev.ctypes.data, hashes.ctypes.data, status.ctypes.data)
    check(rc, "hkv_check_headers", v.lib)
    hb = hashes.tobytes()
    return [hb[32 * i: 32 * i + 32] for i in range(n)], status


def check_headers_device(v, dev: int, d_headers: int, n: int, d_pow_limit: int, d_prev_hash: Optional[int],
                         d_hashes: int, d_status: int, stream: int = 0) -> None:
    """Device-pointer form (HBM-resident header batches; enqueued, not synchronised)."""
    rc = v.lib.hkv_check_headers_device(v.ctx, dev, ctypes.c_void_p(d_headers), n, ctypes.c_void_p(d_pow_limit),
                                        ctypes.c_void_p(d_prev_hash) if d_prev_hash else None,
                                        ctypes.c_void_p(d_hashes), ctypes.c_void_p(d_status),
                                        ctypes.c_void_p(stream) if stream else None)
    check(rc, "hkv_check_headers_device", v.lib)
