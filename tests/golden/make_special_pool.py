"""Generate the committed "special pool" fixture: verify records whose verdict
needs elliptic-curve construction (not a byte mutation), labelled by
construction, for sprinkling into the large adversarial batches
(hkv/adversarial.py, BASELINE configs[3] / configs[4]).

    python tests/golden/make_special_pool.py

Writes ``special_pool.bin`` (n x 168-byte records, include/hkv.h layout) and
``special_pool.json`` (per record: class, label in LIBSECP and HASKOIN mode).
The labels are the construction's intent; the generator asserts them against
the Python restatement, and tests/test_adversarial_labels.py re-checks every
record against the C restatement and OpenSSL (oracle/openssl_check.c).

Classes (SURVEY.md §8(c) known-answer constructions):
  r_plus_n_branch      valid only through the r + n < p retry: R.x in [n, p)
  r_eq_full_x_rejected the same tuple with r = R.x (>= n): compact overflow
  edge_u1 / edge_u2    keyless tuples with u1 / u2 in {1, 2, n-1, n-2, lambda,
                       n-lambda, 2^128-1, 2^128, 2^128+1, 2^129+3, 2^255,
                       n/2, (n+1)/2, 2^32-1}
  u1_zero / u1_zero_msg_n   msg32 = 0 / msg32 = n (msg mod n = 0), valid
  msg_ge_n             msg32 = m + n for a signature of m (reduced mod n), valid
  sum_infinity         u1*G + u2*Q = infinity: reject
  collide_*            ladder collisions (acc = +-T mid-chain) with Q = +-G
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
SEED = 0x53504F4C


# Jacobian scalar multiplication (fast enough for a few hundred fixtures)
def _jdbl(p):
    x, y, z = p
    if y == 0:
        return (0, 1, 0)
    a = x * x % P
    b = y * y % P
    c = b * b % P
    d = 2 * ((x + b) ** 2 - a - c) % P
    e = 3 * a % P
    x3 = (e * e - 2 * d) % P
    return (x3, (e * (d - x3) - 8 * c) % P, 2 * y * z % P)


def _jadd(p, q):
    if p[2] == 0:
        return q
    if q[2] == 0:
        return p
    z1s, z2s = p[2] * p[2] % P, q[2] * q[2] % P
    u1, u2 = p[0] * z2s % P, q[0] * z1s % P
    s1, s2 = p[1] * z2s * q[2] % P, q[1] * z1s * p[2] % P
    if u1 == u2:
        return _jdbl(p) if s1 == s2 else (0, 1, 0)
    h, r = (u2 - u1) % P, (s2 - s1) % P
    h2 = h * h % P
    h3 = h * h2 % P
    v = u1 * h2 % P
    x3 = (r * r - h3 - 2 * v) % P
    return (x3, (r * (v - x3) - s1 * h3) % P, h * p[2] * q[2] % P)


def mul(k: int, pt):
    k %= N
    if pt is None or k == 0:
        return None
    acc, base = (0, 1, 0), (pt[0], pt[1], 1)
    for bit in bin(k)[2:]:
        acc = _jdbl(acc)
        if bit == "1":
            acc = _jadd(acc, base)
    if acc[2] == 0:
        return None
    zi = pow(acc[2], -1, P)
    return (acc[0] * zi * zi % P, acc[1] * zi * zi * zi % P)


def add(a, b):
    return o.point_add(a, b)


def be(x: int) -> bytes:
    return (x % 2**256).to_bytes(32, "big")


def main() -> None:
    rng = random.Random(SEED)
    recs, meta = [], []

    def put(cls, msg, r, s, q_or_pk, compressed=True, label=None):
        pk = q_or_pk if isinstance(q_or_pk, bytes) else o.pubkey_serialize(q_or_pk, compressed)
        rec = o.make_record(msg, be(r) + be(s), pk)
        lib, hask = label
        assert o.verify_record(rec, o.HKV_LIBSECP) == lib, cls
        assert o.verify_record(rec, o.HKV_HASKOIN) == hask, cls
        recs.append(rec)
        meta.append({"class": cls, "libsecp": lib, "haskoin": hask})

    def key():
        return mul(rng.randrange(1, N), G)

    def keyless(q, a, b):
        """R = aG + bQ, r = R.x mod n, s = r/b, msg = a*s; low-S flip keeps it valid."""
        R = add(mul(a, G), mul(b, q))
        r = R[0] % N
        s = r * pow(b, -1, N) % N
        msg = a * s % N
        if s > o.HALF_N:
            s = N - s
        return be(msg), r, s

    VALID, INVALID = (True, True), (False, False)

    # r + n branch: x = n + k with x^3 + 7 a square, R = (x, y); Q = b^-1 (R - aG)
    xr, found = N + 1, []
    while len(found) < 64:
        rhs = (xr ** 3 + 7) % P
        y = pow(rhs, (P + 1) // 4, P)
        if y * y % P == rhs:
            found.append((xr, y if rng.random() < 0.5 else P - y))
        xr += 1 + rng.randrange(3)
    for k, (x, y) in enumerate(found):
        a, b = rng.randrange(1, N), rng.randrange(1, N)
        q = mul(pow(b, -1, N), add((x, y), o.point_neg(mul(a, G))))
        r = x - N
        s = r * pow(b, -1, N) % N
        msg = a * s % N
        if s > o.HALF_N:
            s = N - s
        put("r_plus_n_branch", be(msg), r, s, q, k % 2 == 0, VALID)
        put("r_eq_full_x_rejected", be(msg), x, s, q, k % 2 == 0, INVALID)

    edges = [1, 2, N - 1, N - 2, o.LAMBDA, N - o.LAMBDA, 2**128 - 1, 2**128, 2**128 + 1, 2**129 + 3,
             2**255, N // 2, (N + 1) // 2, 0xFFFFFFFF]
    for rep in range(4):
        for e in edges:
            q = key()
            put("edge_u2", *keyless(q, rng.randrange(1, N), e), q, rep % 2 == 0, label=VALID)
            q = key()
            put("edge_u1", *keyless(q, e, rng.randrange(1, N)), q, rep % 2 == 1, label=VALID)

    for k in range(32):
        q = key()
        b = rng.randrange(1, N)
        R = mul(b, q)
        r = R[0] % N
        s = r * pow(b, -1, N) % N
        if s > o.HALF_N:
            s = N - s
        put("u1_zero", be(0), r, s, q, k % 2 == 0, VALID)
        put("u1_zero_msg_n", be(N), r, s, q, k % 2 == 1, VALID)

    # msg32 >= n: sign m < 2^256 - n with a known key, store m + n
    for k in range(32):
        d = rng.randrange(1, N)
        q = mul(d, G)
        m = rng.randrange(1, 2**256 - N)
        while True:
            kk = rng.randrange(1, N)
            r = mul(kk, G)[0] % N
            s = pow(kk, -1, N) * (m + r * d) % N
            if r and s:
                break
        if s > o.HALF_N:
            s = N - s
        put("msg_ge_n", be(m + N), r, s, q, k % 2 == 0, VALID)

    # sum = infinity: Q = -(a/b) G
    for k in range(32):
        a, b = rng.randrange(1, N), rng.randrange(1, N)
        q = mul((-a * pow(b, -1, N)) % N, G)
        r = rng.randrange(1, N)
        s = r * pow(b, -1, N) % N
        msg = a * s % N
        if s > o.HALF_N:
            s = N - s
        put("sum_infinity", be(msg), r, s, q, k % 2 == 0, INVALID)

    # ladder collisions with Q = +-G (acc == T / acc == -T inside the shared chain)
    for (a, b, qq, cls) in [(1, 1, G, "collide_double_G"), (2, 1, G, "collide_2G_plus_G"),
                            (2, N - 1, G, "collide_cancel_then_add"), (3, 5, G, "q_is_g_small"),
                            (5, 3, o.point_neg(G), "q_is_neg_g"), (2**128, 1, G, "q_is_g_u1_hi"),
                            (1, o.LAMBDA, G, "q_is_g_u2_lambda"), (17, 17, G, "collide_equal_digits"),
                            (2**128 + 1, 2**128 + 1, G, "collide_wide")]:
        for comp in (True, False):
            put(cls, *keyless(qq, a, b), qq, comp, label=VALID)
    for comp in (True, False):  # 1*G + (n-1)*G = infinity
        r = rng.randrange(1, N)
        s = r * pow(N - 1, -1, N) % N
        msg = s % N
        if s > o.HALF_N:
            s = N - s
        put("collide_cancel_to_inf", be(msg), r, s, G, comp, INVALID)

    with open(os.path.join(HERE, "special_pool.bin"), "wb") as f:
        f.write(b"".join(recs))
    with open(os.path.join(HERE, "special_pool.json"), "w") as f:
        json.dump({"seed": SEED, "record_size": o.REC_SIZE, "count": len(recs),
                   "generator": "tests/golden/make_special_pool.py", "records": meta}, f, indent=0)
    print(f"{len(recs)} records; valid {sum(m['libsecp'] for m in meta)}")


if __name__ == "__main__":
    main()
