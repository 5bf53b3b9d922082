"""The construction labels of hkv.adversarial (configs[3] / configs[4]
batches) and of the special-pool fixture agree with two independent
checkers — the C restatement and OpenSSL 3 behind the semantic adapter — on
every class, both modes (CPU)."""
import json
import os
import random

import numpy as np

import secp256k1_oracle as o
from conftest import GOLDEN, openssl_batch, oracle_batch
from hkv import adversarial


def valid_records(n, seed):
    rng = random.Random(seed)
    recs = []
    for i in range(n):
        q = o.point_mul(rng.randrange(1, o.N), o.G)
        m, r, s = o.keyless_tuple(rng.randrange(1, o.N), rng.randrange(1, o.N), q)
        if s > o.N // 2:
            s = o.N - s
        recs.append(o.make_record(m, r.to_bytes(32, "big") + s.to_bytes(32, "big"),
                                  o.pubkey_serialize(q, i % 5 != 0)))
    return np.frombuffer(b"".join(recs), dtype=np.uint8)


def test_special_pool_labels_both_checkers(coracle, openssl):
    """tests/golden/special_pool.bin: every record's manifest label equals the
    C restatement's and OpenSSL's verdict in both modes."""
    data = open(os.path.join(GOLDEN, "special_pool.bin"), "rb").read()
    man = json.load(open(os.path.join(GOLDEN, "special_pool.json")))
    assert len(data) == 168 * man["count"]
    classes = {m["class"] for m in man["records"]}
    assert {"r_plus_n_branch", "r_eq_full_x_rejected", "edge_u1", "edge_u2", "u1_zero", "u1_zero_msg_n",
            "msg_ge_n", "sum_infinity", "collide_cancel_to_inf"} <= classes
    for mode, key in ((0, "libsecp"), (1, "haskoin")):
        exp = np.array([m[key] for m in man["records"]])
        assert (oracle_batch(coracle, data, mode) == exp).all()
        assert (openssl_batch(openssl, data, mode) == exp).all()


def test_labels_match_both_checkers_every_class(coracle, openssl):
    base = valid_records(96, 3)
    assert oracle_batch(coracle, base.tobytes(), 0).all()
    adv, lib, hask, cls = adversarial.mutate(np.tile(base, 40), seed=5, invalid_frac=0.7, special_frac=0.2)
    assert set(np.unique(cls)) == set(range(-1, len(adversarial.CLASSES)))
    for mode, lab in ((0, lib), (1, hask)):
        got_c = oracle_batch(coracle, adv.tobytes(), mode)
        got_o = openssl_batch(openssl, adv.tobytes(), mode)
        bad = sorted({adversarial.CLASSES[c] for c in cls[(got_c != lab) | (got_o != lab)]})
        assert not bad, (mode, bad)
    # each invalid class really is rejected in LIBSECP mode, the valid ones accepted
    for k, (name, l, _) in enumerate(adversarial.INVALID_CLASSES + adversarial.VALID_CLASSES):
        if not name.startswith("special"):
            assert (lib[cls == k] == bool(l)).all(), name


def test_neg_mod_n_matches_python():
    rng = random.Random(9)
    vals = [rng.randrange(1, o.N) for _ in range(200)] + [1, o.N - 1, o.N // 2, 2**64, 2**192 - 1]
    arr = np.frombuffer(b"".join(v.to_bytes(32, "big") for v in vals), dtype=np.uint8).reshape(-1, 32)
    out = adversarial._neg_mod_n(arr)
    assert [int.from_bytes(r.tobytes(), "big") for r in out] == [o.N - v for v in vals]


def test_mutation_is_seeded_and_leaves_input():
    base = valid_records(8, 4)
    keep = base.copy()
    a1 = adversarial.mutate(np.tile(base, 20), 7)[0]
    a2 = adversarial.mutate(np.tile(base, 20), 7)[0]
    assert (a1 == a2).all() and (base == keep).all()


def test_config4_shares():
    """At configs[3] size the shares hold: 30% invalid spread evenly over the
    invalid classes, 5% special valid (labels only; no checker run)."""
    base = valid_records(16, 8)
    n = 1 << 16
    adv, lib, hask, cls = adversarial.mutate(np.tile(base, n // 16), seed=0x484B5634)
    inv = np.isin(cls, np.arange(len(adversarial.INVALID_CLASSES)))
    assert 0.29 < inv.mean() < 0.31
    counts = np.bincount(cls[inv], minlength=len(adversarial.INVALID_CLASSES))
    assert counts.min() > 0.8 * counts.mean()
    assert 0.68 < lib.mean() < 0.72
