"""Generate the committed golden KAT fixtures for the verify path.

    python tests/golden/make_golden.py

Writes ``kat_records.bin`` (n x 168-byte records, include/hkv.h layout) and
``kat_manifest.json`` (per record: class name, expected verdict in LIBSECP and
HASKOIN modes). Expected verdicts come from the Python restatement
(oracle/secp256k1_oracle.py); tests/test_oracle.py re-checks every fixture
against the C restatement and, on the classes where the semantics agree,
against OpenSSL 3.0.2. The constructions are SURVEY.md §8(c)'s known-answer
classes (keyless valid tuples, the r+n branch, sum = infinity, adversarial
encodings, edge scalars, internal-collision cases of the GPU ladder).

Parity note: the reference (haskoin-node) holds no ECDSA vectors, so these
verdicts are pinned by the oracle + OpenSSL cross-check, not by the reference.
"""
from __future__ import annotations

import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import secp256k1_oracle as o  # noqa: E402

N, P, G = o.N, o.P, o.G
SEED = 0x484B5634


def be(x: int) -> bytes:
    return (x % 2**256).to_bytes(32, "big")


def sig(r: int, s: int) -> bytes:
    return be(r) + be(s)


def main() -> None:
    rng = random.Random(SEED)
    recs, meta = [], []

    def add(cls: str, msg: bytes, r: int, s: int, pk: bytes, pklen: int | None = None):
        rec = bytearray(o.make_record(msg, sig(r, s), pk))
        if pklen is not None:
            rec[96] = pklen
        rec = bytes(rec)
        recs.append(rec)
        meta.append({"class": cls,
                     "libsecp": bool(o.verify_record(rec, o.HKV_LIBSECP)),
                     "haskoin": bool(o.verify_record(rec, o.HKV_HASKOIN))})

    def rand_key():
        d = rng.randrange(1, N)
        return o.point_mul(d, G)

    def keyless(q, a=None, b=None):
        a = rng.randrange(1, N) if a is None else a
        b = rng.randrange(1, N) if b is None else b
        return o.keyless_tuple(a, b, q)

    # 1-3: valid, all key encodings
    for k in range(40):
        q = rand_key()
        m, r, s = keyless(q)
        add("valid_compressed", m, r, s, o.pubkey_serialize(q, True))
    for k in range(20):
        q = rand_key()
        m, r, s = keyless(q)
        add("valid_uncompressed", m, r, s, o.pubkey_serialize(q, False))
    for k in range(10):
        q = rand_key()
        m, r, s = keyless(q)
        pk = bytes([6 | (q[1] & 1)]) + o.pubkey_serialize(q, False)[1:]
        add("valid_hybrid", m, r, s, pk)
        bad = bytes([6 | ((q[1] & 1) ^ 1)]) + pk[1:]
        add("hybrid_bad_parity", m, r, s, bad)
    # 5: high-S (LIBSECP rejects, HASKOIN accepts)
    for k in range(20):
        q = rand_key()
        m, r, s = keyless(q)
        add("high_s", m, r, N - s, o.pubkey_serialize(q, k % 2 == 0))
    # 6: r / s range
    q = rand_key()
    m, r, s = keyless(q)
    pk = o.pubkey_serialize(q, True)
    for cls, rr, ss in [("r_zero", 0, s), ("s_zero", r, 0), ("r_eq_n", N, s), ("s_eq_n", r, N),
                        ("r_n_plus_k", N + 7, s), ("r_max", 2**256 - 1, s), ("s_max", r, 2**256 - 1),
                        ("s_n_minus_1", r, N - 1), ("s_half_n", r, o.HALF_N), ("s_half_n_plus_1", r, o.HALF_N + 1)]:
        add(cls, m, rr, ss, pk)
    # 7-10: pubkey encodings
    for k in range(5):
        q = rand_key()
        m, r, s = keyless(q)
        unc = o.pubkey_serialize(q, False)
        off = unc[:33] + be(q[1] + 1)
        add("off_curve_y_plus_1", m, r, s, off)
        add("x_ge_p_compressed", m, r, s, bytes([2]) + be(P + k))
        add("x_max_compressed", m, r, s, bytes([3]) + be(2**256 - 1 - k))
        add("y_ge_p_uncompressed", m, r, s, unc[:33] + be(P + k))
        for pre in (0x00, 0x01, 0x05, 0x08, 0xFF):
            add(f"bad_prefix_{pre:02x}", m, r, s, bytes([pre]) + unc[1:33])
        add("len33_prefix04", m, r, s, bytes([4]) + unc[1:33])
        add("len65_prefix02", m, r, s, bytes([2]) + unc[1:])
        add("len0", m, r, s, b"")
        add("len64", m, r, s, unc[1:])
        add("len_byte_200", m, r, s, o.pubkey_serialize(q, True), pklen=200)
    # non-residue x (compressed) — x = 5 has no point
    q = rand_key()
    m, r, s = keyless(q)
    xs = [x for x in range(1, 60) if pow((x ** 3 + 7) % P, (P - 1) // 2, P) != 1][:6]
    for x in xs:
        add("non_residue_x", m, r, s, bytes([2 + (x & 1)]) + be(x))
    # 11-12: wrong message / wrong key
    for k in range(10):
        q = rand_key()
        m, r, s = keyless(q)
        mb = bytearray(m)
        mb[rng.randrange(32)] ^= 1 << rng.randrange(8)
        add("flipped_msg_bit", bytes(mb), r, s, o.pubkey_serialize(q, True))
        add("wrong_key", m, r, s, o.pubkey_serialize(rand_key(), True))
    # 13: msg >= n (reduced mod n -> valid)
    for k in range(8):
        q = rand_key()
        m, r, s = keyless(q)
        mi = int.from_bytes(m, "big")
        if mi + N < 2**256:
            add("msg_ge_n", be(mi + N), r, s, o.pubkey_serialize(q, True))
    # 14: u1 = 0 (msg = 0 and msg = n)
    for k in range(3):
        q = rand_key()
        m, r, s = keyless(q, a=0)
        add("u1_zero", m, r, s, o.pubkey_serialize(q, True))
        add("u1_zero_msg_n", be(N), r, s, o.pubkey_serialize(q, True))
    # 15: the r + n branch — R.x in [n, p)
    xr = N + 1  # x = n would give r = 0
    found = []
    while len(found) < 4 and xr < P:
        rhs = (xr ** 3 + 7) % P
        y = pow(rhs, (P + 1) // 4, P)
        if y * y % P == rhs:
            found.append((xr, y))
        xr += 1
    for (x, y) in found:
        R = (x, y)
        a, b = rng.randrange(1, N), rng.randrange(1, N)
        aG = o.point_mul(a, G)
        q = o.point_mul(pow(b, -1, N), o.point_add(R, o.point_neg(aG)))
        r = x - N
        s = r * pow(b, -1, N) % N
        msg = a * s % N
        if s > o.HALF_N:  # flip keeps m and yields -R (same x)
            s = N - s
        add("r_plus_n_branch", be(msg), r, s, o.pubkey_serialize(q, True))
        add("r_eq_full_x_rejected", be(msg), x, s, o.pubkey_serialize(q, True))
    # 16: sum = infinity: Q = -(a/b) G
    for k in range(4):
        a, b = rng.randrange(1, N), rng.randrange(1, N)
        q = o.point_mul((-a * pow(b, -1, N)) % N, G)
        r = rng.randrange(1, N)
        s = r * pow(b, -1, N) % N
        msg = a * s % N
        if s > o.HALF_N:
            s = N - s
        add("sum_infinity", be(msg), r, s, o.pubkey_serialize(q, k % 2 == 0))
    # 17: edge scalars (u1, u2) via keyless
    edges = [1, 2, N - 1, N - 2, o.LAMBDA, N - o.LAMBDA, 2**128 - 1, 2**128, 2**128 + 1, 2**129 + 3,
             2**255, N // 2, (N + 1) // 2, 0xFFFFFFFF]
    for u2 in edges:
        q = rand_key()
        m, r, s = keyless(q, b=u2)
        add("edge_u2", m, r, s, o.pubkey_serialize(q, True))
    for u1 in edges:
        q = rand_key()
        m, r, s = keyless(q, a=u1)
        add("edge_u1", m, r, s, o.pubkey_serialize(q, False))
    # 18-19: Q = +-G and ladder collisions (acc == T, acc == -T mid-chain)
    for (a, b, qq, cls) in [(1, 1, G, "collide_double_G"), (2, 1, G, "collide_2G_plus_G"),
                            (1, N - 1, G, "collide_cancel_to_inf"), (2, N - 1, G, "collide_cancel_then_add"),
                            (3, 5, G, "q_is_g_small"), (5, 3, o.point_neg(G), "q_is_neg_g"),
                            (2**128, 1, G, "q_is_g_u1_hi"), (1, o.LAMBDA, G, "q_is_g_u2_lambda"),
                            (17, 17, G, "collide_equal_digits"), (2**128 + 1, 2**128 + 1, G, "collide_wide")]:
        R = o.double_mul(a % N, b % N, qq)
        if R is None or R[0] % N == 0:
            r = rng.randrange(1, N)
            s = r * pow(b, -1, N) % N
            msg = a * s % N
        else:
            msg, r, s = o.keyless_tuple(a, b, qq)
            msg = int.from_bytes(msg, "big")
        if s > o.HALF_N:
            s = N - s
        add(cls, be(msg), r, s, o.pubkey_serialize(qq, True))
    # the reference fixtures' P2PK key (test/Haskoin/NodeSpec.hs:289) as Q
    ref_pk = bytes.fromhex("0304eca640a331eccab38ec13e969fa2ed638ec1dfd4e1e3824ab19f011890af73")
    q = o.pubkey_parse(ref_pk)
    assert q is not None
    for k in range(4):
        m, r, s = keyless(q)
        add("reference_fixture_key", m, r, s, ref_pk)
    # trailing garbage after a 33-byte key is ignored
    q = rand_key()
    m, r, s = keyless(q)
    pk = o.pubkey_serialize(q, True)
    rec = bytearray(o.make_record(m, sig(r, s), pk))
    rec[130:162] = bytes(rng.randrange(256) for _ in range(32))
    recs.append(bytes(rec))
    meta.append({"class": "compressed_trailing_garbage",
                 "libsecp": bool(o.verify_record(bytes(rec), 0)),
                 "haskoin": bool(o.verify_record(bytes(rec), 1))})

    with open(os.path.join(HERE, "kat_records.bin"), "wb") as f:
        f.write(b"".join(recs))
    with open(os.path.join(HERE, "kat_manifest.json"), "w") as f:
        json.dump({"seed": SEED, "record_size": o.REC_SIZE, "count": len(recs),
                   "generator": "tests/golden/make_golden.py", "records": meta}, f, indent=0)
    n_acc = sum(m["libsecp"] for m in meta), sum(m["haskoin"] for m in meta)
    print(f"{len(recs)} records, accepted libsecp={n_acc[0]} haskoin={n_acc[1]}")


if __name__ == "__main__":
    main()
