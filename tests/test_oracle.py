"""CPU tests: pin the oracle before trusting it (no GPU needed).

* curve / GLV constants re-derived from first principles;
* the reference's own fixtures: SHA-256d header hashes asserted by
  /root/reference/test/Haskoin/NodeSpec.hs:180-218 (committed as
  tests/golden/ref_*.{bin,json}) and the fixture coinbase P2PK key;
* golden KAT verdicts == Python restatement == C restatement (both modes);
* cross-check against OpenSSL 3.0.2 ECDSA_do_verify on the classes where
  libsecp256k1 and OpenSSL semantics agree.
"""
import ctypes
import ctypes.util
import json
import os
import random

import pytest

import secp256k1_oracle as o
from conftest import GOLDEN, oracle_batch


def test_curve_constants():
    assert o.on_curve(o.GX, o.GY)
    assert pow(o.BETA, 3, o.P) == 1 and o.BETA != 1
    assert pow(o.LAMBDA, 3, o.N) == 1 and o.LAMBDA != 1
    assert o.point_mul(o.LAMBDA, o.G) == (o.BETA * o.GX % o.P, o.GY)
    for a, b in ((o.A1, o.B1), (o.A2, o.B2)):
        assert (a + b * o.LAMBDA) % o.N == 0
        assert abs(a).bit_length() <= 129 and abs(b).bit_length() <= 129


def test_device_glv_constants_and_bounds():
    """The kernel's GLV split (hkv_scalar.h glv_split) restated on ints."""
    g1 = (2**384 * o.B2 + o.N // 2) // o.N
    g2 = (2**384 * (-o.B1) + o.N // 2) // o.N
    assert g1 == 0x3086D221A7D46BCDE86C90E49284EB153DAA8A1471E8CA7FE893209A45DBB031
    assert g2 == 0xE4437ED6010E88286F547FA90ABFE4C4221208AC9DF506C61571B4AE8AC47F71
    rng = random.Random(5)
    ks = [rng.randrange(o.N) for _ in range(3000)] + [0, 1, o.N - 1, o.LAMBDA, 2**128, 2**255, o.N // 2]
    for k in ks:
        c1 = (k * g1 + 2**383) >> 384
        c2 = (k * g2 + 2**383) >> 384
        k2 = (c1 * (-o.B1) + c2 * (-o.B2)) % o.N
        k1 = (k - k2 * o.LAMBDA) % o.N
        m1 = o.N - k1 if k1 > o.N // 2 else k1
        m2 = o.N - k2 if k2 > o.N // 2 else k2
        assert m1 < 2**129 and m2 < 2**129
        s1 = -1 if k1 > o.N // 2 else 1
        s2 = -1 if k2 > o.N // 2 else 1
        assert (s1 * m1 + s2 * m2 * o.LAMBDA - k) % o.N == 0


def booth(k, w, nwin):
    digits = []
    for i in range(nwin):
        v = ((k << 1) >> (w * i)) & ((1 << (w + 1)) - 1)
        digits.append(((v + 1) >> 1) - ((v >> w) << w))
    return digits


def test_top_window_merge_digit_range():
    """HKV_TOP_MERGE (pair_chain, hkv_ecmult_kernel): the top two radix-16
    windows of a GLV half run as one digit m = 16 d32 + d31, taken from the
    8-entry table as min(m, 8) + (m - 8)+. That needs m in [0, 16] for every
    half: the rounding split bounds |k1| by (|a1| + |a2|) / 2 and |k2| by
    (|b1| + |b2|) / 2, both < 2^128 (a wave with any m outside the range
    would run the windows one by one)."""
    assert (abs(o.A1) + abs(o.A2)) // 2 < 2**128 and (abs(o.B1) + abs(o.B2)) // 2 < 2**128
    rng = random.Random(11)
    g1 = (2**384 * o.B2 + o.N // 2) // o.N
    g2 = (2**384 * (-o.B1) + o.N // 2) // o.N
    ks = [rng.randrange(o.N) for _ in range(3000)] + [0, 1, o.N - 1, o.LAMBDA, 2**128, 2**255, o.N // 2]
    seen_top = 0
    for k in ks:
        c1 = (k * g1 + 2**383) >> 384
        c2 = (k * g2 + 2**383) >> 384
        k2 = (c1 * (-o.B1) + c2 * (-o.B2)) % o.N
        k1 = (k - k2 * o.LAMBDA) % o.N
        for kk in (k1, k2):
            mag = o.N - kk if kk > o.N // 2 else kk
            assert mag < 2**128
            d = booth(mag, 4, 33)
            m = 16 * d[32] + d[31]
            assert 0 <= m <= 16
            e1 = min(m, 8)
            assert 0 <= m - e1 <= 8
            assert (e1 + (m - e1)) * 16**31 + sum(x * 16**i for i, x in enumerate(d[:31])) == mag
            seen_top += d[32] != 0
    assert seen_top > 0  # the case the merge removes a window of doublings for


def test_booth_recoding_identity():
    """Booth digits as the ecmult kernel extracts them: radix 16 (Q windows,
    the default hkv_layout.h HKV_QW = 4: 33 windows of -8..8), radix 32 (the
    measured-and-rejected HKV_QW = 5 knob: 26 windows) — each carries any
    |k| < 2^129 the GLV split produces — and radix 2^20 (G, GTAB_W)."""
    rng = random.Random(9)
    for _ in range(2000):
        k = rng.randrange(2**131)
        d = booth(k, 4, 33)
        assert all(-8 <= x <= 8 for x in d)
        assert sum(x * 16**i for i, x in enumerate(d)) == k
        k = rng.choice([rng.randrange(2**129), 2**129 - 1 - rng.randrange(2**20)])
        d = booth(k, 5, 26)
        assert all(-16 <= x <= 16 for x in d)
        assert sum(x * 32**i for i, x in enumerate(d)) == k
        u = rng.randrange(2**128)
        e = booth(u, 20, 7)                        # GWIN = 7 windows of 20 bits
        assert all(-2**19 <= x <= 2**19 for x in e)
        assert sum(x * 2**(20 * i) for i, x in enumerate(e)) == u
        assert all(abs(x) < 2**20 for x in e)       # fits GD_MAG (20 bits)


def test_reference_fixture_hashes():
    """SHA-256d against the header hashes the reference's tests assert."""
    raw = open(os.path.join(GOLDEN, "ref_blocks.bin"), "rb").read()
    fx = json.load(open(os.path.join(GOLDEN, "ref_fixtures.json")))
    off, hashes = 0, []
    while off < len(raw):
        hdr = raw[off:off + 80]
        hashes.append(o.sha256d(hdr)[::-1].hex())
        off += 80 + 1
        st = off
        off += 4
        nin = raw[off]; off += 1
        for _ in range(nin):
            off += 36; sl = raw[off]; off += 1 + sl + 4
        nout = raw[off]; off += 1
        for _ in range(nout):
            off += 8; sl = raw[off]; off += 1 + sl
        off += 4
        assert o.sha256d(raw[st:off]) == hdr[36:68]  # merkle root of a 1-tx block
    h = fx["hashes"]
    assert hashes[4:6] == h["get_blocks"]          # NodeSpec.hs:180-183
    assert hashes[14] == h["best_h15"]             # :197-198
    assert hashes[9] == h["ancestor_h10"]          # :199-200
    assert hashes[11:14] == h["parents_of_h15"]    # :215-218


def test_reference_fixture_pubkey_parses(coracle):
    pk = bytes.fromhex(json.load(open(os.path.join(GOLDEN, "ref_fixtures.json")))["coinbase_p2pk_pubkey"])
    q = o.pubkey_parse(pk)
    assert q is not None
    out = ctypes.create_string_buffer(64)
    assert coracle.hkvo_pubkey_parse(pk, len(pk), out) == 1
    assert out.raw == q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big")


def test_golden_python_matches_manifest(kat):
    recs, meta = kat
    for rec, m in zip(recs, meta):
        assert o.verify_record(rec, o.HKV_LIBSECP) == m["libsecp"], m["class"]
        assert o.verify_record(rec, o.HKV_HASKOIN) == m["haskoin"], m["class"]


def test_golden_c_oracle_matches_manifest(kat, coracle):
    recs, meta = kat
    data = b"".join(recs)
    for mode, key in ((0, "libsecp"), (1, "haskoin")):
        got = oracle_batch(coracle, data, mode)
        exp = [m[key] for m in meta]
        bad = [meta[i]["class"] for i in range(len(meta)) if bool(got[i]) != exp[i]]
        assert not bad, bad


def test_c_oracle_matches_python_random(coracle):
    rng = random.Random(77)
    recs = []
    for i in range(120):
        q = o.point_mul(rng.randrange(1, o.N), o.G)
        m, r, s = o.keyless_tuple(rng.randrange(1, o.N), rng.randrange(1, o.N), q)
        kind = i % 5
        if kind == 1:
            s = o.N - s
        elif kind == 2:
            m = bytes([m[0] ^ 0x80]) + m[1:]
        elif kind == 3:
            q = o.point_mul(rng.randrange(1, o.N), o.G)
        recs.append(o.make_record(m, r.to_bytes(32, "big") + s.to_bytes(32, "big"),
                                  o.pubkey_serialize(q, i % 3 != 0)))
    data = b"".join(recs)
    for mode in (0, 1):
        got = oracle_batch(coracle, data, mode)
        exp = [o.verify_record(r, mode) for r in recs]
        assert list(map(bool, got)) == exp


# --- OpenSSL 3.0.2 cross-check --------------------------------------------
NID_secp256k1 = 714


def _openssl():
    name = ctypes.util.find_library("crypto")
    if not name:
        pytest.skip("libcrypto not present")
    c = ctypes.CDLL(name)
    vp = ctypes.c_void_p
    for fn, res, args in [
        ("EC_KEY_new_by_curve_name", vp, [ctypes.c_int]),
        ("EC_KEY_get0_group", vp, [vp]),
        ("EC_POINT_new", vp, [vp]),
        ("EC_POINT_free", None, [vp]),
        ("EC_POINT_oct2point", ctypes.c_int, [vp, vp, ctypes.c_char_p, ctypes.c_size_t, vp]),
        ("EC_KEY_set_public_key", ctypes.c_int, [vp, vp]),
        ("EC_KEY_free", None, [vp]),
        ("BN_bin2bn", vp, [ctypes.c_char_p, ctypes.c_int, vp]),
        ("ECDSA_SIG_new", vp, []),
        ("ECDSA_SIG_set0", ctypes.c_int, [vp, vp, vp]),
        ("ECDSA_SIG_free", None, [vp]),
        ("ECDSA_do_verify", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, vp, vp]),
    ]:
        f = getattr(c, fn)
        f.restype = res
        f.argtypes = args
    return c


def openssl_verdict(c, rec: bytes, mode: int) -> bool:
    """OpenSSL with the semantic adapter: OpenSSL accepts high-S (pre-reject
    in LIBSECP mode, normalize in HASKOIN mode); verify <= 0 means reject."""
    msg, r, s = rec[:32], int.from_bytes(rec[32:64], "big"), int.from_bytes(rec[64:96], "big")
    pklen = rec[96]
    pk = rec[97:97 + pklen]
    if r >= o.N or s >= o.N:
        return False
    if s > o.HALF_N:
        if mode == o.HKV_LIBSECP:
            return False
        s = o.N - s
    key = c.EC_KEY_new_by_curve_name(NID_secp256k1)
    grp = c.EC_KEY_get0_group(key)
    pt = c.EC_POINT_new(grp)
    try:
        if c.EC_POINT_oct2point(grp, pt, pk, len(pk), None) != 1:
            return False
        if c.EC_KEY_set_public_key(key, pt) != 1:
            return False
        sig = c.ECDSA_SIG_new()
        br = c.BN_bin2bn(r.to_bytes(32, "big"), 32, None)
        bs = c.BN_bin2bn(s.to_bytes(32, "big"), 32, None)
        c.ECDSA_SIG_set0(sig, br, bs)
        v = c.ECDSA_do_verify(msg, 32, sig, key)
        c.ECDSA_SIG_free(sig)
        return v == 1
    finally:
        c.EC_POINT_free(pt)
        c.EC_KEY_free(key)


# classes where OpenSSL's parser differs from secp256k1_ec_pubkey_parse
OPENSSL_PARSE_DIFFERS = {"len_byte_200", "len0", "bad_prefix_00"}


def test_golden_cross_check_openssl(kat):
    c = _openssl()
    recs, meta = kat
    bad = []
    for rec, m in zip(recs, meta):
        if m["class"] in OPENSSL_PARSE_DIFFERS or rec[96] > 65:
            continue
        for mode, key in ((0, "libsecp"), (1, "haskoin")):
            if openssl_verdict(c, rec, mode) != m[key]:
                bad.append((m["class"], key))
    assert not bad, bad


def test_golden_all_classes_openssl_adapter(kat, openssl):
    """The C OpenSSL checker (oracle/openssl_check.c: length / prefix gate
    before EC_POINT_oct2point, high-S adapter, <= 0 is reject) agrees with
    the manifest on EVERY golden class, the parser-only ones included."""
    from conftest import openssl_batch
    recs, meta = kat
    data = b"".join(recs)
    for mode, key in ((0, "libsecp"), (1, "haskoin")):
        got = openssl_batch(openssl, data, mode)
        bad = [meta[i]["class"] for i in range(len(meta)) if bool(got[i]) != meta[i][key]]
        assert not bad, (key, bad)
