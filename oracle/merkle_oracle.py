"""CPU oracle for block merkle roots — TEST INFRASTRUCTURE ONLY (imported by
tests/ as the checker; never by the product path).

Restates haskoin-core-1.1.0 ``Haskoin.Block.Merkle.buildMerkleRoot`` [dep,
absent from /root/reference; /root/reference/stack.yaml:10], the function the
reference's block test applies (``test/Haskoin/NodeSpec.hs:185-193``:
``b.header.merkle `shouldBe` buildMerkleRoot (ths b)``): each level pairs
adjacent hashes and takes SHA-256d of their 64-byte concatenation, an odd
level's last hash is paired with itself, until one hash is left.
``mutated`` restates Bitcoin Core's ComputeMerkleRoot CVE-2012-2459 flag (two
equal hashes paired at some level).

Pinned by: the 15 reference fixture blocks (their header merkle field equals
the root of their txids, tests/golden/ref_blocks.bin) and mainnet block
100,000 (4 txids, published root), both in tests/test_merkle.py.
"""
from __future__ import annotations

import hashlib
from typing import List, Sequence, Tuple


def dsha256(b: bytes) -> bytes:
    return hashlib.sha256(hashlib.sha256(b).digest()).digest()


def merkle_root(txids: Sequence[bytes]) -> Tuple[bytes, bool]:
    """(root, mutated) for txids in digest (internal) byte order. Empty: zeros."""
    level: List[bytes] = list(txids)
    if not level:
        return bytes(32), False
    mutated = False
    while len(level) > 1:
        for i in range(0, len(level) - 1, 2):
            if level[i] == level[i + 1]:
                mutated = True
        if len(level) % 2:
            level.append(level[-1])
        level = [dsha256(level[i] + level[i + 1]) for i in range(0, len(level), 2)]
    return level[0], mutated
