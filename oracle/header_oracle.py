"""CPU oracle (TEST INFRASTRUCTURE ONLY) — pure-Python restatement of the
header checks haskoin-node's header sync relies on.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker. The product path
(``haskoin-node_amd/``) never imports it.

Call site in the reference: ``importHeaders``
(``/root/reference/src/Haskoin/Node/Chain.hs:500-520``) passes each peer's
headers to haskoin-core ``connectBlocks`` [dep: haskoin-core-1.1.0, pinned at
``/root/reference/stack.yaml:10`` / ``stack.yaml.lock:14-20``; not vendored].
For every header that function computes:

* ``headerHash``  — SHA-256d of the 80-byte wire form
  (``Haskoin.Block.Common``); pinned by the hashes the reference's tests
  assert for the fixture chain (``test/Haskoin/NodeSpec.hs:180-218``).
* ``decodeCompact`` — the compact target (``Haskoin.Block.Common``), the same
  rule as Bitcoin's ``arith_uint256::SetCompact``: size = bits >> 24, word =
  bits & 0x7fffff shifted right by 8*(3-size) when size <= 3; negative when
  word != 0 and bit 0x00800000 is set; overflow when word != 0 and
  (size > 34 or word > 0xff and size > 33 or word > 0xffff and size > 32).
* ``isValidPOW net h`` (``Haskoin.Block.Headers``): false when target <= 0,
  overflow, or target > powLimit; else headerPOW h <= target, where headerPOW
  reads the hash bytes as a little-endian integer.
* the predecessor link: the header's prev field equals the hash of the
  header before it (``connectBlocks`` looks each parent up by that field).

Status flags are the HKV_HDR_* constants of ``include/hkv.h``.
Parity: pinned for headerHash and the accept path by the 15 fixture headers;
the reject flags follow the restated rule above (the fixtures hold no
invalid header), with hand-checked edge cases in tests/test_headers.py.
"""
from __future__ import annotations

import hashlib
from typing import List, Optional, Tuple

POW_OK, LINK_OK, NEGATIVE, OVERFLOW, ZERO_TARGET, ABOVE_LIMIT, HASH_ABOVE = 1, 2, 4, 8, 16, 32, 64

# powLimit of the networks haskoin-core defines (Haskoin.Network.Constants) [dep]
POW_LIMIT = {
    "btc": 0x00000000FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF,
    "btcTest": 0x00000000FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF,
    "btcRegTest": 0x7FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF,
    "bchRegTest": 0x7FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF,
}


def header_hash(hdr: bytes) -> bytes:
    """headerHash: SHA-256d of the 80-byte header, digest byte order."""
    assert len(hdr) == 80
    return hashlib.sha256(hashlib.sha256(hdr).digest()).digest()


def decode_compact(bits: int) -> Tuple[int, bool, bool]:
    """(|target|, negative, overflow) — haskoin-core decodeCompact."""
    size = bits >> 24
    word = bits & 0x007FFFFF
    if size <= 3:
        word >>= 8 * (3 - size)
        value = word
    else:
        value = word << (8 * (size - 3))
    neg = word != 0 and (bits & 0x00800000) != 0
    over = word != 0 and (size > 34 or (word > 0xFF and size > 33) or (word > 0xFFFF and size > 32))
    return value, neg, over


def pow_flags(hdr: bytes, pow_limit: int) -> int:
    h = int.from_bytes(header_hash(hdr), "little")
    bits = int.from_bytes(hdr[72:76], "little")
    value, neg, over = decode_compact(bits)
    fl = 0
    if neg:
        fl |= NEGATIVE
    if over:
        fl |= OVERFLOW
    if value == 0:
        fl |= ZERO_TARGET
    if not over:
        if value > pow_limit:
            fl |= ABOVE_LIMIT
        if h > value:
            fl |= HASH_ABOVE
    if not fl:
        fl |= POW_OK
    return fl


def is_valid_pow(hdr: bytes, pow_limit: int) -> bool:
    return bool(pow_flags(hdr, pow_limit) & POW_OK)


def check_headers(headers: List[bytes], pow_limit: int,
                  prev_hash: Optional[bytes] = None) -> Tuple[List[bytes], List[int]]:
    """Per header: (headerHash, HKV_HDR_* flags) — the hkv_check_headers contract."""
    hashes = [header_hash(h) for h in headers]
    status = []
    for i, h in enumerate(headers):
        fl = pow_flags(h, pow_limit)
        want = hashes[i - 1] if i else prev_hash
        if want is None or h[4:36] == want:
            fl |= LINK_OK
        status.append(fl)
    return hashes, status


def encode_compact(value: int) -> int:
    """Inverse used by the test generators (Bitcoin GetCompact, non-negative)."""
    size = (value.bit_length() + 7) // 8
    if size <= 3:
        word = value << (8 * (3 - size))
    else:
        word = value >> (8 * (size - 3))
    if word & 0x00800000:
        word >>= 8
        size += 1
    return (size << 24) | word
