"""The synthetic-batch contract behind BASELINE configs[4] (CPU): the C
restatement of hkv_gen_batch_device (oracle/hkv_oracle.c hkvo_gen_batch) —
record k of batch `seed` depends on (seed, k) only, so contiguous slices
generated independently (one per rank) are the one-process batch; the
construction labels equal the C restatement's and OpenSSL's verdicts in both
modes; every mutation class occurs and rejects. The GPU generator is checked
byte for byte against this restatement in tests/test_gpu_parity.py."""
import numpy as np
import pytest

from conftest import c_gen_batch, openssl_batch, oracle_batch

SEED4 = 0x484B5635  # BASELINE configs[4]


def test_slices_concatenate_to_the_batch(coracle):
    whole, lab, cls = c_gen_batch(coracle, SEED4, 0, 1200, 64, 100, 50)
    parts = []
    for lo, hi in ((0, 64), (64, 577), (577, 1200)):
        r, l2, c2 = c_gen_batch(coracle, SEED4, lo, hi - lo, 64, 100, 50)
        assert (l2 == lab[lo:hi]).all() and (c2 == cls[lo:hi]).all()
        parts.append(r)
    assert (np.concatenate(parts) == whole).all()


def test_zero_invalid_is_the_plain_generator(coracle):
    """invalid_permille = 0 draws nothing extra: the valid records are the
    same as in the mutated batch wherever the latter kept them."""
    plain, lab0, cls0 = c_gen_batch(coracle, SEED4, 0, 800, 64, 100, 0)
    mixed, lab, cls = c_gen_batch(coracle, SEED4, 0, 800, 64, 100, 50)
    assert lab0.all() and (cls0 == -1).all()
    p, m = plain.reshape(-1, 168), mixed.reshape(-1, 168)
    assert (p[lab] == m[lab]).all()
    assert (p[~lab] != m[~lab]).any(axis=1).all()


@pytest.mark.parametrize("permille", [50, 400])
def test_labels_equal_both_checkers_both_modes(coracle, openssl, permille):
    n = 2500
    recs, lab, cls = c_gen_batch(coracle, SEED4 + permille, 0, n, 256, 100, permille)
    frac = 1 - lab.mean()
    assert abs(frac - permille / 1000) < 0.04
    assert set(np.unique(cls[cls >= 0])) == {0, 1, 2, 3, 4}
    for mode in (0, 1):
        assert (oracle_batch(coracle, recs.tobytes(), mode, threads=8) == lab).all()
        assert (openssl_batch(openssl, recs.tobytes(), mode, threads=8) == lab).all()


def test_uncompressed_share_and_negated_keys(coracle):
    recs, lab, cls = c_gen_batch(coracle, 7, 0, 3000, 32, 300, 200)
    r = recs.reshape(-1, 168)
    unc = r[:, 96] == 65
    assert 0.25 < unc.mean() < 0.35
    assert set(np.unique(r[~unc, 97])) <= {2, 3} and (r[unc, 97] == 4).all()
    neg = cls == 4
    assert neg.any() and not lab[neg].any()


def test_blockgen_ripemd160_published_vectors():
    """hkv.blockgen's RIPEMD-160 (the multisig generator's P2SH hashes)
    against the published test vectors and the oracle's restatement."""
    import os
    import sighash_oracle as sh
    from hkv.blockgen import ripemd160
    assert ripemd160(b"").hex() == "9c1185a5c5e9fc54612808977ee8f548b2258d31"
    assert ripemd160(b"abc").hex() == "8eb208f7e05d987a9b044a8e98c6b087f15a0bfc"
    assert ripemd160(b"message digest").hex() == "5d0689ef49d2fae572b881b123a85ffa21595f36"
    for n in (55, 56, 64, 119, 120, 300):
        d = os.urandom(n)
        assert ripemd160(d) == sh.ripemd160(d)
