"""Adversarial record batches with verdicts known by construction
(BASELINE configs[3] and the 5%-invalid configs[4] IBD batch; SURVEY.md §8(c)
"Adversarial classes for config 4").

Starting from valid records (the keyless construction of hkv_gen_records_kernel),
a seeded share ``invalid_frac`` (30%) is mutated evenly into the invalid
classes below and a share ``special_frac`` (5%) into the special valid
classes. Every class has a verdict fixed by the reference semantics, so a
batch of any size carries exact labels without a checker run over it
(tests/test_adversarial_labels.py checks every class against the C
restatement and OpenSSL):

  class               mutation                                 LIBSECP HASKOIN rule
  msg_bit             flip one bit of msg32                     reject  reject  a3 (9)-(11)
  r_zero / s_zero     r = 0 / s = 0                             reject  reject  a3 (4)
  r_eq_n / s_eq_n     r = n / s = n                             reject  reject  a5 overflow
  r_n_plus_k          r = n + k, 0 < k < 2^32                   reject  reject  a5 overflow
  r_max / s_max       r = 2^256 - 1 / s = 2^256 - 1             reject  reject  a5 overflow
  bad_prefix          prefix in {00, 01, 05, 08, ff}            reject  reject  a4
  prefix_flip         prefix ^= 04 (02/03 -> 06/07 at 33 B ...)  reject  reject  a4 length/prefix
  x_ge_p              33-byte key, x = p + k or 2^256 - 1 - k   reject  reject  a4 range
  y_ge_p              65-byte 04 key, y = p + k                 reject  reject  a4 range
  off_curve           65-byte 04 key, y + 1                     reject  reject  a4 on-curve
  non_residue_x       33-byte key, x^3 + 7 not a square         reject  reject  a4 sqrt
  hybrid_bad_parity   65-byte 06/07 key, parity(y) mismatch     reject  reject  a4 hybrid
  len_mismatch        02/03 with length 65, 04 with length 33   reject  reject  a4 length
  wrong_q             another record's key                      reject  reject  a3 (9)-(11)
  special_invalid     sum = inf, r = R.x >= n, cancel-to-inf    reject  reject  a3 (8), a5
  high_s              s = n - s                                 reject  accept  a3 (1) vs a1
  -- valid --
  reencode            02/03 <-> 04 (same point)                 accept  accept  a4
  valid_hybrid        65-byte 06/07 key, correct parity         accept  accept  a4 hybrid
  special_valid       r + n branch, edge u1/u2, u1 = 0, msg32   accept  accept  a3 (3), (10)
                      >= n, ladder collisions (pool)

The "special" records need elliptic-curve construction rather than a byte
mutation; they come from the committed fixture tests/golden/special_pool.bin
(tests/golden/make_special_pool.py, labels asserted against the oracle there
and re-checked in the tests). msg_bit and wrong_q are rejects except with
probability ~2^-256. Record layout: include/hkv.h (msg32 | r | s | pklen |
pubkey[65] | pad, 168 B).
"""
from __future__ import annotations

import json
import os
from typing import Tuple

import numpy as np

N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
P = 2**256 - 2**32 - 977
REC = 168

# (name, LIBSECP verdict, HASKOIN verdict)
INVALID_CLASSES = (("msg_bit", 0, 0), ("r_zero", 0, 0), ("s_zero", 0, 0), ("r_eq_n", 0, 0), ("s_eq_n", 0, 0),
                   ("r_n_plus_k", 0, 0), ("r_max", 0, 0), ("s_max", 0, 0), ("bad_prefix", 0, 0),
                   ("prefix_flip", 0, 0), ("x_ge_p", 0, 0), ("y_ge_p", 0, 0), ("off_curve", 0, 0),
                   ("non_residue_x", 0, 0), ("hybrid_bad_parity", 0, 0), ("len_mismatch", 0, 0),
                   ("wrong_q", 0, 0), ("special_invalid", 0, 0), ("high_s", 0, 1))
VALID_CLASSES = (("reencode", 1, 1), ("valid_hybrid", 1, 1), ("special_valid", 1, 1))
CLASSES = tuple(c[0] for c in INVALID_CLASSES + VALID_CLASSES)
_CID = {c: i for i, c in enumerate(CLASSES)}

POOL_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests", "golden",
                         "special_pool.bin")


def _be(x: int) -> np.ndarray:
    return np.frombuffer((x % 2**256).to_bytes(32, "big"), dtype=np.uint8)


def _neg_mod_n(s_be: np.ndarray) -> np.ndarray:
    """n - s for rows of 32 big-endian bytes (0 < s < n)."""
    w = s_be.copy().view(">u8").astype(np.uint64)  # [k, 4] big-endian words, word 0 most significant
    nw = np.array([(N >> (64 * (3 - i))) & 0xFFFFFFFFFFFFFFFF for i in range(4)], dtype=np.uint64)
    out = np.zeros_like(w)
    borrow = np.zeros(w.shape[0], dtype=np.uint64)
    for i in (3, 2, 1, 0):
        a = nw[i]
        out[:, i] = a - w[:, i] - borrow  # wraps mod 2^64
        borrow = ((w[:, i] > a) | ((w[:, i] == a) & (borrow == 1))).astype(np.uint64)
    return out.astype(">u8").view(np.uint8).reshape(-1, 32)


def _words_plus(base: int, k: np.ndarray) -> np.ndarray:
    """Rows of 32 big-endian bytes of base + k, for uint64 k whose add does not
    carry out of the low 64-bit word (base's low word + k < 2^64, or k wraps
    the low word of 2^256 - 1 downwards)."""
    w = np.array([(base >> (64 * (3 - q))) & 0xFFFFFFFFFFFFFFFF for q in range(4)], dtype=np.uint64)
    out = np.tile(w, (k.size, 1))
    out[:, 3] = w[3] + k.astype(np.uint64)
    return out.astype(">u8").view(np.uint8).reshape(-1, 32)


def _y_of(rec: np.ndarray) -> int:
    """The y coordinate of a (valid, 02/03/04-encoded) record's key."""
    x = int.from_bytes(rec[98:130].tobytes(), "big")
    if rec[96] == 65:
        return int.from_bytes(rec[130:162].tobytes(), "big")
    y = pow((x * x * x + 7) % P, (P + 1) // 4, P)
    return y if (y & 1) == (rec[97] & 1) else P - y


def _non_residue_xs(rng: np.random.Generator, k: int) -> list:
    out = []
    while len(out) < k:
        x = int.from_bytes(rng.bytes(32), "big") % P
        if pow((x ** 3 + 7) % P, (P - 1) // 2, P) == P - 1:
            out.append(x)
    return out


def load_pool(path: str = POOL_PATH) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(records [k, 168], LIBSECP labels, HASKOIN labels) of the special pool."""
    raw = np.fromfile(path, dtype=np.uint8).reshape(-1, REC)
    man = json.load(open(os.path.splitext(path)[0] + ".json"))
    lib = np.array([m["libsecp"] for m in man["records"]], dtype=bool)
    hask = np.array([m["haskoin"] for m in man["records"]], dtype=bool)
    assert len(lib) == raw.shape[0]
    return raw, lib, hask


def mutate(records: np.ndarray, seed: int, invalid_frac: float = 0.30, special_frac: float = 0.05,
           pool_path: str = POOL_PATH, twin: np.ndarray | None = None
           ) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """Returns (records', label_libsecp, label_haskoin, cls) for a flat uint8
    array of valid records; cls is -1 for untouched records, else an index
    into CLASSES. The input array is not modified.

    twin: optionally the same records with every key in 65-byte form (the
    device generator with the same seed and uncompressed_permille = 1000
    picks the same keys and scalars), so the classes that need y read it
    instead of taking a square root per compressed key on the host."""
    orig = records.reshape(-1, REC)
    tw = None if twin is None else twin.reshape(-1, REC)
    a = orig.copy()
    n = a.shape[0]
    rng = np.random.default_rng(seed)
    cls = np.full(n, -1, dtype=np.int16)
    u = rng.random(n)
    hit = np.nonzero(u < invalid_frac)[0]
    cls[hit] = rng.integers(0, len(INVALID_CLASSES), size=hit.size)
    sp = np.nonzero((u >= invalid_frac) & (u < invalid_frac + special_frac))[0]
    cls[sp] = len(INVALID_CLASSES) + rng.integers(0, len(VALID_CLASSES), size=sp.size)
    sel = lambda name: np.nonzero(cls == _CID[name])[0]  # noqa: E731
    comp = orig[:, 96] == 33

    i = sel("msg_bit")
    a[i, rng.integers(0, 32, i.size)] ^= (1 << rng.integers(0, 8, i.size)).astype(np.uint8)
    a[sel("r_zero"), 32:64] = 0
    a[sel("s_zero"), 64:96] = 0
    a[sel("r_eq_n"), 32:64] = _be(N)
    a[sel("s_eq_n"), 64:96] = _be(N)
    i = sel("r_n_plus_k")
    a[i, 32:64] = _words_plus(N, 1 + rng.integers(0, 2**32 - 1, i.size, dtype=np.uint64))
    a[sel("r_max"), 32:64] = 0xFF
    a[sel("s_max"), 64:96] = 0xFF
    i = sel("bad_prefix")
    a[i, 97] = np.array([0x00, 0x01, 0x05, 0x08, 0xFF], dtype=np.uint8)[rng.integers(0, 5, i.size)]
    a[sel("prefix_flip"), 97] ^= 0x04
    i = sel("x_ge_p")
    k = rng.integers(0, 2**32, i.size, dtype=np.uint64)
    a[i, 98:130] = np.where((rng.random(i.size) < 0.5)[:, None], _words_plus(P, k),
                            _words_plus(2**256 - 1, ~k + np.uint64(1)))
    a[i, 96], a[i, 97] = 33, 2 + rng.integers(0, 2, i.size).astype(np.uint8)
    a[i, 130:162] = 0
    for name in ("y_ge_p", "off_curve", "hybrid_bad_parity", "valid_hybrid", "reencode"):
        for j in sel(name):
            y = _y_of(orig[j]) if tw is None else int.from_bytes(tw[j, 130:162].tobytes(), "big")
            if name == "reencode" and not comp[j]:
                a[j, 96], a[j, 97] = 33, 2 | (y & 1)
                a[j, 130:162] = 0
                continue
            a[j, 96] = 65
            a[j, 97] = 4
            if name == "y_ge_p":
                y = P + int(rng.integers(0, 2**32))
            elif name == "off_curve":
                y = (y + 1) % P
            elif name == "hybrid_bad_parity":
                a[j, 97] = 6 | ((y & 1) ^ 1)
            elif name == "valid_hybrid":
                a[j, 97] = 6 | (y & 1)
            a[j, 130:162] = _be(y)
    i = sel("non_residue_x")
    if i.size:
        xs = _non_residue_xs(rng, 64)
        for j in i:
            a[j, 96], a[j, 97] = 33, 2 + int(rng.integers(0, 2))
            a[j, 98:130] = _be(xs[int(rng.integers(0, len(xs)))])
            a[j, 130:162] = 0
    i = sel("len_mismatch")
    a[i, 96] = np.where(comp[i], 65, 33).astype(np.uint8)
    i = sel("wrong_q")
    if i.size and n > 1:  # a donor record whose key has another x
        don = (i + 1 + rng.integers(0, n - 1, i.size)) % n
        for q in np.nonzero((orig[don, 98:130] == orig[i, 98:130]).all(axis=1))[0]:
            while (orig[don[q], 98:130] == orig[i[q], 98:130]).all():
                don[q] = (don[q] + 1) % n
        a[i, 96:162] = orig[don, 96:162]
    i = sel("high_s")
    if i.size:
        a[i, 64:96] = _neg_mod_n(a[i, 64:96])
    lib = np.ones(n, dtype=bool)
    hask = np.ones(n, dtype=bool)
    for k, (name, l, h) in enumerate(INVALID_CLASSES + VALID_CLASSES):
        if name.startswith("special"):
            continue
        lib[cls == k] = bool(l)
        hask[cls == k] = bool(h)
    si, sv = sel("special_invalid"), sel("special_valid")
    if si.size or sv.size:
        pool, plib, phask = load_pool(pool_path)
        for idx, want in ((si, False), (sv, True)):
            cand = np.nonzero(plib == want)[0]
            pick = cand[rng.integers(0, cand.size, idx.size)]
            a[idx] = pool[pick]
            lib[idx] = plib[pick]
            hask[idx] = phask[pick]
    return a.reshape(-1), lib, hask, cls


def unpack_bits(words: np.ndarray, n: int) -> np.ndarray:
    return np.unpackbits(words.astype(np.uint32).view(np.uint8), bitorder="little")[:n].astype(bool)
