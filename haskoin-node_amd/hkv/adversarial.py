"""Adversarial record batches with verdicts known by construction
(BASELINE configs[3] and the 5%-invalid configs[4] IBD batch; SURVEY.md §8(c)
"Adversarial classes for config 4").

Starting from valid records (the keyless construction of hkv_gen_records_kernel),
a seeded fraction is mutated into one invalid class each. Every class has a
verdict fixed by the reference semantics, so a batch of any size carries exact
labels without running a checker over it:

  class            mutation                          LIBSECP  HASKOIN  reference rule
  msg_bit          flip one bit of msg32             reject   reject   a3 (9)-(11): R.x no longer matches
  r_zero           r = 0                             reject   reject   a3 (4)
  s_overflow       s = 2^256 - 1 (>= n)              reject   reject   a5 compact parse overflow
  bad_prefix       pubkey prefix ^= 0x04             reject   reject   a4 (02/03 -> 06/07 with 33 B, 04 -> 00)
  x_ge_p           pubkey x = 2^256 - 1 (>= p)       reject   reject   a4 range check
  high_s           s = n - s                         reject   accept   a3 (1) vs a1 normalizeSig then verify

The msg_bit class is rejected except with probability ~2^-256 (the flipped
message would have to produce the same u1·G + u2·Q x-coordinate mod n).
Record layout: include/hkv.h (msg32 ‖ r ‖ s ‖ pklen ‖ pubkey[65] ‖ pad, 168 B).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
REC = 168
CLASSES = ("msg_bit", "r_zero", "s_overflow", "bad_prefix", "x_ge_p", "high_s")
_N_WORDS = np.array([(N >> (64 * (3 - i))) & 0xFFFFFFFFFFFFFFFF for i in range(4)], dtype=np.uint64)


def _neg_mod_n(s_be: np.ndarray) -> np.ndarray:
    """n - s for rows of 32 big-endian bytes (0 < s < n)."""
    w = s_be.copy().view(">u8").astype(np.uint64)  # [k, 4] big-endian words, word 0 most significant
    out = np.zeros_like(w)
    borrow = np.zeros(w.shape[0], dtype=np.uint64)
    for i in (3, 2, 1, 0):
        a = _N_WORDS[i]
        d = a - w[:, i] - borrow  # wraps mod 2^64
        borrow = ((w[:, i] > a) | ((w[:, i] == a) & (borrow == 1))).astype(np.uint64)
        out[:, i] = d
    return out.astype(">u8").view(np.uint8).reshape(-1, 32)


def mutate(records: np.ndarray, seed: int, invalid_frac: float = 0.30
           ) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """Returns (records', label_libsecp, label_haskoin, cls) for a flat uint8
    array of valid records; cls is -1 for untouched records, else an index
    into CLASSES. The input array is not modified."""
    a = records.reshape(-1, REC).copy()
    n = a.shape[0]
    rng = np.random.default_rng(seed)
    cls = np.full(n, -1, dtype=np.int8)
    hit = np.nonzero(rng.random(n) < invalid_frac)[0]
    cls[hit] = rng.integers(0, len(CLASSES), size=hit.size)
    sel = lambda k: np.nonzero(cls == k)[0]  # noqa: E731
    i = sel(0)
    a[i, rng.integers(0, 32, i.size)] ^= (1 << rng.integers(0, 8, i.size)).astype(np.uint8)
    a[sel(1), 32:64] = 0
    a[sel(2), 64:96] = 0xFF
    a[sel(3), 97] ^= 0x04
    a[sel(4), 98:130] = 0xFF
    i = sel(5)
    if i.size:
        a[i, 64:96] = _neg_mod_n(a[i, 64:96])
    lib = cls < 0
    hask = (cls < 0) | (cls == 5)
    return a.reshape(-1), lib, hask, cls


def unpack_bits(words: np.ndarray, n: int) -> np.ndarray:
    return np.unpackbits(words.astype(np.uint32).view(np.uint8), bitorder="little")[:n].astype(bool)
