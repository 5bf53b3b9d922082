"""CPU oracle (TEST INFRASTRUCTURE ONLY) — pure-Python restatement of the
reference hot path's verify semantics.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker. The product path
(``haskoin-node_amd/``) never imports it.

What it restates. None of these functions lives in
``/root/reference``: they are un-vendored dependencies pinned at
``/root/reference/stack.yaml:8-10`` / ``stack.yaml.lock:7-20``
(haskoin-core-1.1.0, secp256k1-haskell-1.2.0 -> libsecp256k1, nix package
``secp256k1``, version unpinned, ``stack.yaml:2-7``):

* ``pubkey_parse``      — libsecp256k1 ``secp256k1_ec_pubkey_parse`` /
  ``secp256k1_eckey_pubkey_parse`` (a4): 33-byte 02/03 compressed, 65-byte
  04 uncompressed and 06/07 hybrid keys; x, y < p; on-curve; hybrid parity.
* ``sig_parse_compact`` — ``secp256k1_ecdsa_signature_parse_compact`` (a5):
  r or s >= n is an overflow -> parse failure; zero parses.
* ``sig_normalize``     — ``secp256k1_ecdsa_signature_normalize`` (a6).
* ``ecdsa_verify``      — ``secp256k1_ecdsa_verify`` ->
  ``secp256k1_ecdsa_sig_verify`` (a3): reject high-S; m = msg32 mod n;
  reject r == 0 or s == 0; R = (m/s)G + (r/s)Q; reject R = inf; accept if
  R.x == r (mod p as integers), else accept if r + n < p and R.x == r + n.
* ``verify_hash_sig``   — haskoin-core ``Haskoin.Crypto.Signature.verifyHashSig``
  (a1): normalize to low-S FIRST, then verify (so high-S is accepted).

Parity status: the reference's own fixtures
(``test/Haskoin/NodeSpec.hs:282-340``) contain no signatures, so ECDSA verdict
parity is UNPINNED by the reference. This oracle is cross-checked against
OpenSSL 3.0.2 ``ECDSA_do_verify`` on the classes where the semantics agree
(``tests/test_oracle.py``) and against first-principles known-answer
constructions. The one reference-held datum on this path is
the P2PK public key of the fixture coinbases (``NodeSpec.hs:289``), which must
parse.
"""
from __future__ import annotations

import hashlib
from typing import Optional, Tuple

# --- curve constants -------------------------------------------------------
P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8
G = (GX, GY)
HALF_N = N // 2
# GLV endomorphism: lambda*(x, y) = (beta*x, y). Derived (tests/test_oracle.py
# re-derives them as non-trivial cube roots of unity and checks the pairing).
LAMBDA = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72
BETA = 0x7AE96A2B657C07106E64479EAC3434E99CF0497512F58995C1396C28719501EE
# short lattice basis of {(a, b): a + b*lambda = 0 mod n} (extended Euclid)
A1 = 0x3086D221A7D46BCDE86C90E49284EB15
B1 = -0xE4437ED6010E88286F547FA90ABFE4C3
A2 = 0x114CA50F7A8E2F3F657C1108D9D44CFD8
B2 = A1

Point = Optional[Tuple[int, int]]  # None = point at infinity

HKV_LIBSECP = 0  # raw secp256k1_ecdsa_verify: high-S rejected
HKV_HASKOIN = 1  # verifyHashSig: normalize then verify


def on_curve(x: int, y: int) -> bool:
    return (y * y - x * x * x - 7) % P == 0


def point_add(a: Point, b: Point) -> Point:
    if a is None:
        return b
    if b is None:
        return a
    if a[0] == b[0]:
        if (a[1] + b[1]) % P == 0:
            return None
        lam = 3 * a[0] * a[0] * pow(2 * a[1], -1, P) % P
    else:
        lam = (b[1] - a[1]) * pow(b[0] - a[0], -1, P) % P
    x = (lam * lam - a[0] - b[0]) % P
    return (x, (lam * (a[0] - x) - a[1]) % P)


def point_neg(a: Point) -> Point:
    return None if a is None else (a[0], (-a[1]) % P)


def point_mul(k: int, a: Point) -> Point:
    r: Point = None
    for bit in bin(k % N)[2:]:
        r = point_add(r, r)
        if bit == "1":
            r = point_add(r, a)
    return r


def double_mul(u1: int, u2: int, q: Point) -> Point:
    """u1*G + u2*Q by Shamir's trick (affine)."""
    gq = point_add(G, q)
    r: Point = None
    for i in range(255, -1, -1):
        r = point_add(r, r)
        b1, b2 = (u1 >> i) & 1, (u2 >> i) & 1
        if b1 and b2:
            r = point_add(r, gq)
        elif b1:
            r = point_add(r, G)
        elif b2:
            r = point_add(r, q)
    return r


# --- parsing (a4, a5, a6) --------------------------------------------------

def pubkey_parse(data: bytes) -> Point:
    """secp256k1_ec_pubkey_parse semantics. Returns affine point or None."""
    if len(data) == 33 and data[0] in (2, 3):
        x = int.from_bytes(data[1:33], "big")
        if x >= P:
            return None
        rhs = (x * x * x + 7) % P
        y = pow(rhs, (P + 1) // 4, P)
        if y * y % P != rhs:
            return None
        if (y & 1) != (data[0] & 1):
            y = P - y
        return (x, y)
    if len(data) == 65 and data[0] in (4, 6, 7):
        x = int.from_bytes(data[1:33], "big")
        y = int.from_bytes(data[33:65], "big")
        if x >= P or y >= P:
            return None
        if data[0] in (6, 7) and (y & 1) != (data[0] & 1):
            return None
        if not on_curve(x, y):
            return None
        return (x, y)
    return None


def pubkey_serialize(q: Tuple[int, int], compressed: bool = True) -> bytes:
    x, y = q
    if compressed:
        return bytes([2 | (y & 1)]) + x.to_bytes(32, "big")
    return b"\x04" + x.to_bytes(32, "big") + y.to_bytes(32, "big")


def sig_parse_compact(sig64: bytes) -> Optional[Tuple[int, int]]:
    """secp256k1_ecdsa_signature_parse_compact: overflow (>= n) fails."""
    if len(sig64) != 64:
        return None
    r = int.from_bytes(sig64[:32], "big")
    s = int.from_bytes(sig64[32:], "big")
    if r >= N or s >= N:
        return None
    return (r, s)


def sig_normalize(r: int, s: int) -> Tuple[int, int, bool]:
    """secp256k1_ecdsa_signature_normalize: s > n/2 -> n - s."""
    if s > HALF_N:
        return r, N - s, True
    return r, s, False


# --- verify (a3, a1) -------------------------------------------------------

def ecdsa_sig_verify(msg32: bytes, r: int, s: int, q: Point) -> bool:
    """secp256k1_ecdsa_sig_verify (no high-S check)."""
    if q is None or r == 0 or s == 0:
        return False
    m = int.from_bytes(msg32, "big") % N
    sinv = pow(s, -1, N)
    u1 = m * sinv % N
    u2 = r * sinv % N
    R = double_mul(u1, u2, q)
    if R is None:
        return False
    x = R[0]
    if x == r:
        return True
    if r + N < P and x == r + N:
        return True
    return False


def ecdsa_verify(msg32: bytes, r: int, s: int, q: Point) -> bool:
    """secp256k1_ecdsa_verify: rejects high-S, then sig_verify."""
    if s > HALF_N:
        return False
    return ecdsa_sig_verify(msg32, r, s, q)


def verify_hash_sig(msg32: bytes, r: int, s: int, q: Point) -> bool:
    """haskoin-core verifyHashSig: normalize (low-S) then verify."""
    r, s, _ = sig_normalize(r, s)
    return ecdsa_verify(msg32, r, s, q)


# --- the batch record (include/hkv.h) --------------------------------------
REC_SIZE = 168  # msg32 | r32 | s32 | pklen u8 | pubkey[65] | pad[6]


def make_record(msg32: bytes, sig64: bytes, pubkey: bytes) -> bytes:
    assert len(msg32) == 32 and len(sig64) == 64 and len(pubkey) <= 65
    rec = msg32 + sig64 + bytes([len(pubkey)]) + pubkey.ljust(65, b"\0")
    return rec.ljust(REC_SIZE, b"\0")


def verify_record(rec: bytes, mode: int) -> bool:
    """Verdict for one raw record: pubkey parse + compact parse
    (+ normalize in HASKOIN mode) + verify — exactly the CPU harness of
    SURVEY.md §8(d)."""
    msg32 = rec[0:32]
    sig = sig_parse_compact(rec[32:96])
    pklen = rec[96]
    if pklen > 65:
        return False
    q = pubkey_parse(rec[97:97 + pklen])
    if sig is None or q is None:
        return False
    r, s = sig
    if mode == HKV_HASKOIN:
        return verify_hash_sig(msg32, r, s, q)
    return ecdsa_verify(msg32, r, s, q)


# --- helpers used by the KAT constructions ---------------

def keyless_tuple(a: int, b: int, q: Tuple[int, int]) -> Tuple[bytes, int, int]:
    """Valid (msg32, r, s) for pubkey q without a secret key: R = aG + bQ,
    r = R.x mod n, s = r/b, msg = a*s. Returns low-S form (s -> n-s keeps
    validity since x(-R) = x(R))."""
    R = double_mul(a % N, b % N, q)
    assert R is not None
    r = R[0] % N
    assert r != 0
    s = r * pow(b, -1, N) % N
    m = a * s % N
    if s > HALF_N:
        # (m, r, n-s) verifies with u1' = -a, u2' = -b -> -R, same x
        s = N - s
    return m.to_bytes(32, "big"), r, s


def glv_split(k: int) -> Tuple[int, int]:
    """k = k1 + k2*lambda (mod n), |k1|, |k2| ~ 2^128 (signed ints)."""
    c1 = (B2 * k + N // 2) // N
    c2 = (-B1 * k + N // 2) // N
    k1 = k - c1 * A1 - c2 * A2
    k2 = -c1 * B1 - c2 * B2
    return k1, k2


def sha256d(data: bytes) -> bytes:
    return hashlib.sha256(hashlib.sha256(data).digest()).digest()
