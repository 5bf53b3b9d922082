"""Record packing for the batch ABI (include/hkv.h record layout).

The Haskell-side equivalents are secp256k1-haskell ``exportCompactSig`` (r||s)
and ``exportPubKey`` (SEC1 bytes) [dep]; the record simply concatenates the
Hash256 bytes (``msg32``), the compact signature and the serialized key.
"""
from __future__ import annotations

from typing import Iterable, Sequence, Tuple

import numpy as np

from .lib import HKV_RECORD_SIZE


def make_record(msg32: bytes, sig64: bytes, pubkey: bytes) -> bytes:
    if len(msg32) != 32:
        raise ValueError("msg32 must be 32 bytes")
    if len(sig64) != 64:
        raise ValueError("compact signature must be 64 bytes")
    if len(pubkey) > 65:
        raise ValueError("pubkey longer than 65 bytes")
    rec = msg32 + sig64 + bytes([len(pubkey)]) + pubkey.ljust(65, b"\0")
    return rec.ljust(HKV_RECORD_SIZE, b"\0")


def pack_records(items: Iterable[Tuple[bytes, bytes, bytes]]) -> np.ndarray:
    """(msg32, sig64, pubkey) tuples -> contiguous uint8 array [n, 168]."""
    recs = [make_record(m, s, p) for (m, s, p) in items]
    if not recs:
        return np.zeros((0, HKV_RECORD_SIZE), dtype=np.uint8)
    return np.frombuffer(b"".join(recs), dtype=np.uint8).reshape(-1, HKV_RECORD_SIZE).copy()


def unpack_bits(words: np.ndarray, n: int) -> np.ndarray:
    """Verdict bitmap (bit i of word i//32) -> bool[n]."""
    w = np.ascontiguousarray(words, dtype=np.uint32)
    bits = np.unpackbits(w.view(np.uint8), bitorder="little")
    return bits[:n].astype(bool)


def bits_from_bools(v: Sequence[bool]) -> np.ndarray:
    b = np.packbits(np.asarray(v, dtype=np.uint8), bitorder="little")
    pad = (-len(b)) % 4
    return np.frombuffer(b.tobytes() + b"\0" * pad, dtype=np.uint32).copy()
