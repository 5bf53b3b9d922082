"""The construction labels of hkv.adversarial (configs[3] / configs[4]
batches) agree with the oracle on every class, both modes (CPU)."""
import random

import numpy as np

import secp256k1_oracle as o
from conftest import oracle_batch
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


def test_labels_match_oracle_every_class(coracle):
    base = valid_records(96, 3)
    assert oracle_batch(coracle, base.tobytes(), 0).all()
    adv, lib, hask, cls = adversarial.mutate(np.tile(base, 8), seed=5, invalid_frac=0.6)
    assert set(np.unique(cls)) == set(range(-1, len(adversarial.CLASSES)))
    assert (oracle_batch(coracle, adv.tobytes(), 0) == lib).all()
    assert (oracle_batch(coracle, adv.tobytes(), 1) == hask).all()


def test_neg_mod_n_matches_python():
    rng = random.Random(9)
    vals = [rng.randrange(1, o.N) for _ in range(200)] + [1, o.N - 1, o.N // 2, 2**64, 2**192 - 1]
    arr = np.frombuffer(b"".join(v.to_bytes(32, "big") for v in vals), dtype=np.uint8).reshape(-1, 32)
    out = adversarial._neg_mod_n(arr)
    assert [int.from_bytes(r.tobytes(), "big") for r in out] == [o.N - v for v in vals]


def test_mutation_is_seeded_and_leaves_input():
    base = valid_records(8, 4)
    keep = base.copy()
    a1 = adversarial.mutate(base, 7)[0]
    a2 = adversarial.mutate(base, 7)[0]
    assert (a1 == a2).all() and (base == keep).all()
