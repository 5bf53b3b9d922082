"""GPU parity tests (MI355X): the HIP path through the C ABI against the
oracle — bit-exact verdicts, both modes, golden KATs, random and adversarial
batches, field/scalar known answers, determinism, the 1M-record size."""
import ctypes
import os
import random

import numpy as np
import pytest

import secp256k1_oracle as o
from conftest import fast_batch, host_threads, openssl_batch, oracle_batch

pytestmark = pytest.mark.gpu

HKV_DBG = dict(FE_MUL=1, FE_SQR=2, FE_ADD=3, FE_SUB=4, FE_INV=5, FE_SQRT=6, SC_MUL=7, SC_INV=8, GLV=9,
               ECMULT_G=10, MUL512=11, SQR512=12)


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need the MI355X"
    return t


@pytest.fixture(scope="module")
def ver(torch):
    import hkv
    v = hkv.Verifier(hkv.VerifierConfig(device_ids=[0], flags=1))  # HKV_OPEN_NO_SELFCHECK
    yield v
    v.close()


def test_open_with_self_check(torch):
    import hkv
    with hkv.Verifier(hkv.VerifierConfig(device_ids=[0])) as v:
        assert v.num_devices == 1


def limbs(x):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)]


def from_limbs(ws):
    return sum(int(w) << (32 * i) for i, w in enumerate(ws))


def run_debug(torch, ver, op, xs, ys):
    n = len(xs)
    a = torch.tensor(np.array([limbs(x) for x in xs], dtype=np.uint32).view(np.int32), device="cuda")
    b = torch.tensor(np.array([limbs(y) for y in ys], dtype=np.uint32).view(np.int32), device="cuda")
    out = torch.zeros((n, 16), dtype=torch.int32, device="cuda")
    ver.debug_op(0, HKV_DBG[op], n, a.data_ptr(), b.data_ptr(), out.data_ptr())
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def rand_vals(rng, n):
    edge = [0, 1, 2, o.P - 1, o.P, o.P + 1, 2**256 - 1, 2**256 - 2, 2**255, 2**32 + 977, o.N - 1, o.N,
            2**224 - 1, (2**256 - 1) ^ (2**32)]
    return edge + [rng.randrange(2**256) for _ in range(n - len(edge))]


def test_field_ops_known_answers(torch, ver):
    rng = random.Random(1)
    xs, ys = rand_vals(rng, 4096), rand_vals(rng, 4096)[::-1]
    for op, f in [("FE_MUL", lambda x, y: x * y % o.P), ("FE_SQR", lambda x, y: x * x % o.P),
                  ("FE_ADD", lambda x, y: (x + y) % o.P), ("FE_SUB", lambda x, y: (x - y) % o.P)]:
        out = run_debug(torch, ver, op, xs, ys)
        for i in range(len(xs)):
            assert from_limbs(out[i, :8]) == f(xs[i], ys[i]), (op, hex(xs[i]), hex(ys[i]))


def test_mul512_product(torch, ver):
    """Raw 256x256 -> 512-bit limb product (the inline-asm product scanner)."""
    rng = random.Random(7)
    xs, ys = rand_vals(rng, 4096), rand_vals(rng, 4096)[::-1]
    xs += [2**256 - 1] * 4
    ys += [2**256 - 1, 1, 0, 2**255]
    out = run_debug(torch, ver, "MUL512", xs, ys)
    for i in range(len(xs)):
        assert from_limbs(list(out[i, :8])) + (from_limbs(list(out[i, 8:16])) << 256) == xs[i] * ys[i]
    out = run_debug(torch, ver, "SQR512", xs, ys)
    for i in range(len(xs)):
        assert from_limbs(list(out[i, :8])) + (from_limbs(list(out[i, 8:16])) << 256) == xs[i] * xs[i]


def test_field_inv_sqrt(torch, ver):
    rng = random.Random(2)
    xs = [1, 2, 7, o.P - 1] + [rng.randrange(1, o.P) for _ in range(1020)]
    inv = run_debug(torch, ver, "FE_INV", xs, xs)
    sq = run_debug(torch, ver, "FE_SQRT", xs, xs)
    for i, x in enumerate(xs):
        assert from_limbs(inv[i, :8]) == pow(x, o.P - 2, o.P)
        assert from_limbs(sq[i, :8]) == pow(x, (o.P + 1) // 4, o.P)


def test_scalar_ops(torch, ver):
    rng = random.Random(3)
    xs = [1, 2, o.N - 1, o.N // 2] + [rng.randrange(1, o.N) for _ in range(2044)]
    ys = [o.N - 1, o.N - 2, 1, 3] + [rng.randrange(o.N) for _ in range(2044)]
    mul = run_debug(torch, ver, "SC_MUL", xs, ys)
    inv = run_debug(torch, ver, "SC_INV", xs, ys)
    for i in range(len(xs)):
        assert from_limbs(mul[i, :8]) == xs[i] * ys[i] % o.N
        assert from_limbs(inv[i, :8]) == pow(xs[i], o.N - 2, o.N)


def test_glv_split(torch, ver):
    rng = random.Random(4)
    ks = [0, 1, o.N - 1, o.LAMBDA, 2**128, 2**255, o.N // 2] + [rng.randrange(o.N) for _ in range(2041)]
    out = run_debug(torch, ver, "GLV", ks, ks)
    for i, k in enumerate(ks):
        k1 = from_limbs(list(out[i, :5]) + [0, 0, 0])
        k2 = from_limbs(list(out[i, 5:10]) + [0, 0, 0])
        fl = int(out[i, 10])
        assert fl & 4 == 0
        s1 = -1 if fl & 1 else 1
        s2 = -1 if fl & 2 else 1
        assert k1 < 2**129 and k2 < 2**129
        assert (s1 * k1 + s2 * k2 * o.LAMBDA - k) % o.N == 0


def test_ecmult_g_table_source(torch, ver):
    ks = [1, 2, 3, 128, 2**128, 5 * 2**128, o.N - 1]
    out = run_debug(torch, ver, "ECMULT_G", ks, ks)
    for i, k in enumerate(ks):
        q = o.point_mul(k, o.G)
        assert from_limbs(out[i, :8]) == q[0] and from_limbs(out[i, 8:16]) == q[1]


def test_golden_kat_both_modes(ver, kat):
    recs, meta = kat
    arr = np.frombuffer(b"".join(recs), dtype=np.uint8)
    for mode, key in ((0, "libsecp"), (1, "haskoin")):
        got = ver.verify_records(arr, mode)
        bad = [(i, meta[i]["class"]) for i in range(len(meta)) if bool(got[i]) != meta[i][key]]
        assert not bad, (key, bad)


def test_golden_kat_every_offset(ver, kat):
    """Each KAT record at every lane position of a wave (ballot/bitmap path)."""
    recs, meta = kat
    sel = [i for i, m in enumerate(meta) if m["class"] in (
        "valid_compressed", "high_s", "r_plus_n_branch", "sum_infinity", "collide_double_G",
        "collide_cancel_to_inf", "u1_zero", "valid_hybrid")]
    rng = random.Random(5)
    order = [rng.choice(sel) for _ in range(64 * 37 + 5)]
    arr = np.frombuffer(b"".join(recs[i] for i in order), dtype=np.uint8)
    for mode, key in ((0, "libsecp"), (1, "haskoin")):
        got = ver.verify_records(arr, mode)
        exp = np.array([meta[i][key] for i in order])
        assert (got == exp).all()


@pytest.mark.parametrize("n", [(1 << 15) + 256, 139264])
def test_golden_kat_full_grid_yfree(ver, kat, n):
    """Every golden KAT class through the full-grid (y-free) launches: the
    KATs repeated in random order to 33,024 records (the mid-size paired-form
    ecmult instance) and 139,264 (the plain 4-wave instance) — above the split
    bound, so the prologue leaves w = x^3 + 7 and hkv_finish_kernel /
    hkv_rare_kernel / hkv_yverdict_kernel decide — each verdict equal to its
    label in both modes. Covers the rare paths (u1 = 0, sum = infinity,
    u1 G = +-u2 Q collisions), non-residue and off-curve keys, and the r + n
    candidate."""
    recs, meta = kat
    rng = random.Random(11)
    order = list(range(len(recs))) * (n // len(recs)) + [rng.randrange(len(recs)) for _ in range(n % len(recs))]
    rng.shuffle(order)
    arr = np.frombuffer(b"".join(recs[i] for i in order), dtype=np.uint8)
    for mode, key in ((0, "libsecp"), (1, "haskoin")):
        got = ver.verify_records(arr, mode)
        exp = np.array([meta[i][key] for i in order])
        bad = sorted({meta[order[j]]["class"] for j in np.nonzero(got != exp)[0]})
        assert not bad, (key, bad)


def mixed_batch(rng, n):
    recs = []
    for i in range(n):
        q = o.point_mul(rng.randrange(1, o.N), o.G)
        m, r, s = o.keyless_tuple(rng.randrange(1, o.N), rng.randrange(1, o.N), q)
        kind = rng.randrange(8)
        if kind == 1:
            s = o.N - s
        elif kind == 2:
            m = bytes([m[0] ^ 1]) + m[1:]
        elif kind == 3:
            r = (r + 1) % o.N
        recs.append(o.make_record(m, r.to_bytes(32, "big") + s.to_bytes(32, "big"),
                                  o.pubkey_serialize(q, i % 4 != 0)))
    return b"".join(recs)


def test_random_mixed_vs_c_oracle(ver, coracle):
    data = mixed_batch(random.Random(6), 1500)
    for mode in (0, 1):
        exp = oracle_batch(coracle, data, mode, threads=16)
        got = ver.verify_records(np.frombuffer(data, dtype=np.uint8), mode)
        assert (got == exp).all(), np.nonzero(got != exp)


def gen_device(torch, ver, n, seed, unc=100, pool=65536):
    d = torch.empty(n * 168, dtype=torch.uint8, device="cuda")
    ver.gen_records_device(0, seed, n, pool, unc, d.data_ptr())
    torch.cuda.synchronize()
    return d


def gen_twin(torch, ver, d, n, seed):
    """The same generated records with every key in 65-byte form (same seed,
    uncompressed_permille = 1000): the y source of hkv.adversarial.mutate."""
    t = gen_device(torch, ver, n, seed=seed, unc=1000).cpu().numpy()
    a, b = d.cpu().numpy().reshape(-1, 168), t.reshape(-1, 168)
    assert (a[:, :96] == b[:, :96]).all() and (a[:, 98:130] == b[:, 98:130]).all()
    comp = a[:, 96] == 33
    assert ((a[comp, 97] & 1) == (b[comp, 161] & 1)).all()  # prefix parity == y parity
    return t


def test_generated_valid_batch_all_accept_and_oracle_agrees(torch, ver, coracle):
    n = 65536 + 17
    d = gen_device(torch, ver, n, seed=0x484B5632)
    host = d.cpu().numpy()
    got = ver.verify_records(host, 0)
    assert got.all(), int((~got).sum())
    # the generator's records are valid per the independent oracle (sample)
    exp = oracle_batch(coracle, host[: 4096 * 168].tobytes(), 0, threads=16)
    assert exp.all()


def test_adversarial_batch_vs_oracle(torch, ver, coracle, openssl):
    """131,072 records, 30% invalid over every hkv.adversarial class (plus 5%
    special valids): GPU == C restatement == OpenSSL, both modes."""
    from hkv import adversarial
    n = 131072
    d = gen_device(torch, ver, n, seed=0x484B5634, unc=100)
    twin = gen_twin(torch, ver, d, n, 0x484B5634)
    adv, lab_lib, lab_hask, cls = adversarial.mutate(d.cpu().numpy(), seed=11, twin=twin)
    for mode, lab in ((0, lab_lib), (1, lab_hask)):
        exp = oracle_batch(coracle, adv.tobytes(), mode, threads=host_threads())
        got = ver.verify_records(adv, mode)
        mism = np.nonzero(got != exp)[0]
        assert mism.size == 0, (mode, mism[:20], [adversarial.CLASSES[c] for c in cls[mism[:20]]])
        assert (exp == lab).all()
        sl = slice(0, 16384 * 168)
        assert (openssl_batch(openssl, adv[sl].tobytes(), mode, threads=host_threads()) == got[:16384]).all()


def test_device_path_and_determinism(torch, ver):
    n = 1 << 20  # BASELINE config 2 size
    d = gen_device(torch, ver, n, seed=0x484B5632)
    bits = torch.zeros((n + 31) // 32, dtype=torch.int32, device="cuda")
    ver.verify_device(0, d.data_ptr(), n, 0, bits.data_ptr())
    torch.cuda.synchronize()
    b1 = bits.cpu().numpy().view(np.uint32).copy()
    assert (b1 == 0xFFFFFFFF).all()
    bits.zero_()
    ver.verify_device(0, d.data_ptr(), n, 0, bits.data_ptr())
    torch.cuda.synchronize()
    assert (bits.cpu().numpy().view(np.uint32) == b1).all()


def test_odd_sizes(ver, kat):
    recs, meta = kat
    for n in (1, 2, 63, 64, 65, 255, 257):
        sel = [(i * 7) % len(recs) for i in range(n)]
        arr = np.frombuffer(b"".join(recs[i] for i in sel), dtype=np.uint8)
        got = ver.verify_records(arr, 1)
        assert (got == np.array([meta[i]["haskoin"] for i in sel])).all()
    assert ver.verify_records(np.zeros(0, dtype=np.uint8), 0).size == 0


def test_batch_api_pinned_buffer(ver, kat):
    recs, meta = kat
    lib = ver.lib
    b = ctypes.c_void_p()
    assert lib.hkv_batch_alloc(ver.ctx, len(recs), ctypes.byref(b)) == 0
    try:
        buf = lib.hkv_batch_records(b)
        ctypes.memmove(buf, b"".join(recs), len(recs) * 168)
        words = (ctypes.c_uint32 * ((len(recs) + 31) // 32))()
        assert lib.hkv_verify(ver.ctx, b, len(recs), 1, words) == 0
        got = np.unpackbits(np.frombuffer(bytes(words), dtype=np.uint8), bitorder="little")[:len(recs)]
        assert (got.astype(bool) == np.array([m["haskoin"] for m in meta])).all()
        assert lib.hkv_verify(ver.ctx, b, len(recs) + 1, 1, words) == -1  # over capacity
    finally:
        lib.hkv_batch_free(b)


def verify_dev_bits(torch, ver, d, n, mode, offset=0):
    words = torch.zeros((n + 63) // 64 * 2, dtype=torch.int32, device="cuda")
    ver.verify_device(0, d.data_ptr() + offset * 168, n, mode, words.data_ptr())
    torch.cuda.synchronize()
    return words.cpu().numpy().view(np.uint32)


def test_config4_adversarial_1m_both_modes(torch, ver, coracle, openssl):
    """BASELINE configs[3]: 1,048,576 records, 30% invalid spread evenly over
    every SURVEY §8(c) class hkv.adversarial builds (msg bit, r/s in {0, n,
    n+k, 2^256-1}, bad / flipped prefixes, x >= p, y >= p, off-curve,
    non-residue x, hybrid parity, 33/65 length mismatch, wrong Q, sum = inf,
    r = R.x >= n, high-S) plus 5% special valids (re-encoded and hybrid keys,
    the r + n branch, edge u1 / u2, u1 = 0, msg32 >= n, ladder collisions).
    The GPU bitmap must equal, in both modes and on EVERY record, the
    construction labels, the C restatement and OpenSSL's ECDSA_do_verify
    behind the semantic adapter (round 6: every record, was a 262,144-record
    slice)."""
    from hkv import adversarial
    n = 1 << 20
    d = gen_device(torch, ver, n, seed=0x484B5634)
    twin = gen_twin(torch, ver, d, n, 0x484B5634)
    adv, lab_lib, lab_hask, cls = adversarial.mutate(d.cpu().numpy(), seed=0x484B5634, twin=twin)
    assert 0.29 < np.isin(cls, np.arange(len(adversarial.INVALID_CLASSES))).mean() < 0.31
    d.copy_(torch.from_numpy(adv))
    th = host_threads()
    for mode, lab in ((0, lab_lib), (1, lab_hask)):
        got = adversarial.unpack_bits(verify_dev_bits(torch, ver, d, n, mode), n)
        mism = np.nonzero(got != lab)[0]
        assert mism.size == 0, (mode, mism[:10], [adversarial.CLASSES[c] for c in cls[mism[:10]]])
        exp = oracle_batch(coracle, adv.tobytes(), mode, threads=th)
        mism = np.nonzero(got != exp)[0]
        assert mism.size == 0, (mode, "C oracle", mism[:10])
        ossl = openssl_batch(openssl, adv.tobytes(), mode, threads=th)
        mism = np.nonzero(got != ossl)[0]
        assert mism.size == 0, (mode, "openssl", mism[:10])


def gen_batch_dev(torch, ver, seed, index0, n, unc=100, pool=65536, inv=50):
    d = torch.empty(n * 168, dtype=torch.uint8, device="cuda")
    lab = torch.zeros((n + 63) // 64 * 2, dtype=torch.int32, device="cuda")
    ver.gen_batch_device(0, seed, index0, n, pool, unc, inv, d.data_ptr(), lab.data_ptr())
    torch.cuda.synchronize()
    return d, lab.cpu().numpy().view(np.uint32)


def test_gen_batch_matches_c_restatement(torch, ver, coracle):
    """hkv_gen_batch_device == the C restatement (oracle/hkv_oracle.c
    hkvo_gen_batch) byte for byte, labels included, at index 0 and at a
    slice deep inside a 16M batch; invalid_permille = 0 is the plain
    generator (hkv_gen_records_device)."""
    from conftest import c_gen_batch
    from hkv import adversarial
    for seed, index0, n, pool, inv in ((0x484B5635, 0, 1500, 64, 50), (0x484B5635, 9_999_937, 777, 64, 300),
                                       (0x484B5632, 123_456, 500, 65536, 0)):
        d, lab = gen_batch_dev(torch, ver, seed, index0, n, pool=pool, inv=inv)
        recs, clab, cls = c_gen_batch(coracle, seed, index0, n, pool, 100, inv)
        got = d.cpu().numpy()
        bad = np.nonzero((got.reshape(-1, 168) != recs.reshape(-1, 168)).any(axis=1))[0]
        assert bad.size == 0, (seed, index0, bad[:10], cls[bad[:10]])
        assert (adversarial.unpack_bits(lab, n) == clab).all()
    plain = gen_device(torch, ver, 4096, seed=0x484B5632).cpu().numpy()
    d, lab = gen_batch_dev(torch, ver, 0x484B5632, 0, 4096, inv=0)
    assert (d.cpu().numpy() == plain).all() and adversarial.unpack_bits(lab, 4096).all()


@pytest.mark.timeout(1500)
def test_config5_ibd_16m_sharded_bitmap(torch, ver, coracle, secpfast):
    """BASELINE configs[4] exactly as bench.py runs it at N = 8, on one GPU:
    16,777,216 records (seed 0x484B5635, 5% invalid), each of the 8 shards
    (hkv/shard.py) GENERATED on its own with index0 = lo — as each rank does —
    and byte-equal to the same slice of the one-launch batch; the shards'
    verdict words assembled as the all-gather does equal the single-launch
    bitmap and the construction labels bit for bit; a sample of every shard
    equals the C restatement's verdicts: 65,536 records per shard, and EVERY
    record of every shard (mode LIBSECP, the bench's; HASKOIN on 262,144 per
    shard, every record with HKV_FULL_16M=2) equals the libsecp256k1-class
    restatement (oracle/secp_fast.c) — north_star's "zero verdict mismatches
    on 16M mixed valid/invalid signatures" against a checker rather than the
    construction labels (profiles/r06n/ ran both modes on every record in
    70 s on the GPU box's 16 host threads; HKV_FULL_16M=0 keeps only a
    2,048-record sample)."""
    from hkv import adversarial
    from hkv.shard import assemble_bitmap, shard_bounds, words_per_rank
    full_check = os.environ.get("HKV_FULL_16M", "1") not in ("", "0")
    n, world, seed = 1 << 24, 8, 0x484B5635
    d, lab = gen_batch_dev(torch, ver, seed, 0, n)
    labels = adversarial.unpack_bits(lab, n)
    assert 0.045 < 1 - labels.mean() < 0.055
    whole = verify_dev_bits(torch, ver, d, n, 0)[: (n + 31) // 32]
    wpr = words_per_rank(n, world)
    gathered = np.zeros(world * wpr, dtype=np.uint32)
    for r in range(world):
        lo, hi = shard_bounds(n, r, world)
        ds, ls = gen_batch_dev(torch, ver, seed, lo, hi - lo)
        assert torch.equal(ds, d[lo * 168: hi * 168]), r
        assert (adversarial.unpack_bits(ls, hi - lo) == labels[lo:hi]).all()
        w = verify_dev_bits(torch, ver, ds, hi - lo, 0)
        gathered[r * wpr: r * wpr + w.size] = w
        k = 65536 if full_check else 2048
        exp = oracle_batch(coracle, ds[:k * 168].cpu().numpy().tobytes(), 0, threads=host_threads())
        assert (adversarial.unpack_bits(w, k) == exp).all(), r
        if full_check:
            host = ds.cpu().numpy()
            for mode in (0, 1):
                # mode 0 (the bench's) on every record, mode 1 on the first
                # 262,144 of each shard (HKV_FULL_16M=2: every record too)
                m = hi - lo if mode == 0 or os.environ.get("HKV_FULL_16M") == "2" else 262144
                wm = w if mode == 0 else verify_dev_bits(torch, ver, ds, hi - lo, 1)
                exp = fast_batch(secpfast, host[: m * 168], mode, threads=host_threads())
                mism = np.nonzero(adversarial.unpack_bits(wm, m) != exp)[0]
                assert mism.size == 0, (r, mode, "secp_fast", mism[:10])
                print(f"shard {r} mode {mode}: {m} records equal to secp_fast, {int(exp.sum())} accepted",
                      flush=True)
            del host
        del ds
    full = assemble_bitmap(n, world, gathered, wpr)
    assert (full == whole).all()
    got = adversarial.unpack_bits(full, n)
    assert (got == labels).all(), np.nonzero(got != labels)[0][:10]


def test_split_lane_ecmult_matches_full_grid(torch, ver, coracle):
    """Three launch shapes on the same adversarial records: at most 16
    signatures per CU (4,096 on an MI355X) the block kernel
    (hkv_block_kernel<false>: each chain's windows split between the table of
    Q' and that of 2^92 Q'); up to an eighth of the resident grid (32,768)
    the pair kernel (hkv_pair_split_kernel<false>: k1 and k2 chains on their
    own waves, two lanes per chain); above it one lane per signature
    (hkv_ecmult_kernel + the finish kernels). Identical verdicts, equal to
    the labels and to the C oracle on a slice, in both modes; the block
    shape also at a size that is not a multiple of 16 or 32."""
    from hkv import adversarial
    n_blk, n_small, n_big = 1 << 12, 1 << 15, (1 << 15) + 257   # block / pair (32,768) / full grid (33,024)
    d = gen_device(torch, ver, n_big, seed=0x53504C54)
    adv, lab_lib, lab_hask, _ = adversarial.mutate(d.cpu().numpy(), seed=0x53504C54)
    d.copy_(torch.from_numpy(adv))
    for mode, lab in ((0, lab_lib), (1, lab_hask)):
        blk = adversarial.unpack_bits(verify_dev_bits(torch, ver, d, n_blk, mode), n_blk)
        odd = adversarial.unpack_bits(verify_dev_bits(torch, ver, d, n_blk - 37, mode), n_blk - 37)
        small = adversarial.unpack_bits(verify_dev_bits(torch, ver, d, n_small, mode), n_small)
        big = adversarial.unpack_bits(verify_dev_bits(torch, ver, d, n_big, mode), n_big)
        assert (small == big[:n_small]).all()
        assert (blk == big[:n_blk]).all() and (odd == big[:n_blk - 37]).all()
        assert (big == lab).all() and (small == lab[:n_small]).all()
        exp = oracle_batch(coracle, adv[: 8192 * 168].tobytes(), mode, threads=16)
        assert (small[:8192] == exp).all()


def test_host_path_pipelined_chunks_match_device_path(torch, ver):
    """hkv_verify_host over 600,000 records is pipelined in grid-sized chunks
    (H2D of chunk c+1 on the copy stream while chunk c verifies; here
    262,144 + 262,144 + 75,712): the verdict bitmap equals the HBM-resident
    path's, with 1% of the records corrupted so both verdicts occur."""
    n = 600_000
    d = gen_device(torch, ver, n, seed=0x484F5354)
    host = d.cpu().numpy().copy()
    rng = np.random.default_rng(9)
    bad = rng.choice(n, size=n // 100, replace=False)
    host[bad * 168 + 5] ^= 0x40                       # flip a msg32 bit: ECDSA rejects
    d.copy_(torch.from_numpy(host))
    dev = adversarial_unpack(verify_dev_bits(torch, ver, d, n, 0), n)
    got = ver.verify_records(host, 0)
    assert (got == dev).all()
    assert not got[bad].any() and got.sum() == n - bad.size


def adversarial_unpack(words, n):
    from hkv import adversarial
    return adversarial.unpack_bits(words, n)


def test_two_device_contexts_on_one_gpu_match_single(torch, ver):
    """hkv_open_devices([0, 0]): the in-process multi-device path of
    hkv_verify (hkv_api.cpp verify_from_host: contiguous 64-aligned shards,
    per-device copy / verify streams, H2D pipelined in grid-sized chunks, the
    per-shard verdict words merged into the caller's bitmap) exercised with
    two device contexts on one GPU. n = 5 * 2^18 + 17 gives each shard three
    chunks (262,144 + 262,144 + 131,136 / + 131,153) and a ragged last word;
    2% of the records are corrupted."""
    import hkv
    n = 5 * (1 << 18) + 17
    d = gen_device(torch, ver, n, seed=0x4D554C54)
    host = d.cpu().numpy().copy()
    rng = np.random.default_rng(12)
    bad = rng.choice(n, size=n // 50, replace=False)
    host[bad * 168 + 40] ^= 0x01                       # a bit of r: ECDSA rejects
    single = ver.verify_records(host, 0)
    with hkv.Verifier(hkv.VerifierConfig(device_ids=[0, 0], flags=1)) as v2:
        assert v2.num_devices == 2
        for mode in (0, 1):
            got = v2.verify_records(host, mode)
            assert (got == single).all(), np.nonzero(got != single)[0][:10]
    assert not single[bad].any() and single.sum() == n - bad.size


def test_scratch_ordered_across_streams(torch, ver):
    """Device-form calls on two different streams share the device's scratch
    (intermediate, Q tables, verdict words): each call waits for the previous
    call's work (include/hkv.h, Streams), so back-to-back verifies of two
    different batches on two streams each get their own verdicts."""
    n = 200_000
    a = gen_device(torch, ver, n, seed=0x53545231)
    b = a.clone()
    b.view(-1, 168)[::3, 5] ^= 0x20                   # every third record of b rejects
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    wa = torch.zeros((n + 63) // 64 * 2, dtype=torch.int32, device="cuda")
    wb = torch.zeros_like(wa)
    torch.cuda.synchronize()
    for _ in range(3):
        ver.verify_device(0, a.data_ptr(), n, 0, wa.data_ptr(), s1.cuda_stream)
        ver.verify_device(0, b.data_ptr(), n, 0, wb.data_ptr(), s2.cuda_stream)
    torch.cuda.synchronize()
    from hkv import adversarial
    ga = adversarial.unpack_bits(wa.cpu().numpy().view(np.uint32), n)
    gb = adversarial.unpack_bits(wb.cpu().numpy().view(np.uint32), n)
    assert ga.all()
    exp = np.ones(n, dtype=bool)
    exp[::3] = False
    assert (gb == exp).all()


def test_multi_device_failover_reshards(torch, ver):
    """SURVEY §5 failover of the host-batch path (hkv_plan.h
    run_with_failover through hkv_verify_host): three device contexts on one
    GPU; device 1's shard fails before it is enqueued and device 2's after
    its work ran (hkv_debug_fail_device). Both are marked unhealthy, their
    shards are re-verified on device 0, and the bitmap equals the
    single-device one; the next call uses device 0 only; when device 0 fails
    too the call returns HKV_E_HIP, and every later call HKV_E_NODEV."""
    import hkv
    from hkv.lib import HkvError
    n = 3 * (1 << 18) + 4321
    d = gen_device(torch, ver, n, seed=0x46414C4C)
    host = d.cpu().numpy().copy()
    rng = np.random.default_rng(13)
    bad = rng.choice(n, size=n // 40, replace=False)
    host[bad * 168 + 70] ^= 0x10                       # a bit of s: rejects
    single = ver.verify_records(host, 1)
    with hkv.Verifier(hkv.VerifierConfig(device_ids=[0, 0, 0], flags=1)) as v3:
        lib = v3.lib
        assert lib.hkv_debug_fail_device(v3.ctx, 1, 1) == 0   # HKV_FAIL_ENQUEUE
        assert lib.hkv_debug_fail_device(v3.ctx, 2, 2) == 0   # HKV_FAIL_JOIN
        got = v3.verify_records(host, 1)
        assert (got == single).all(), np.nonzero(got != single)[0][:10]
        assert [lib.hkv_device_healthy(v3.ctx, k) for k in range(3)] == [1, 0, 0]
        assert [lib.hkv_device_failures(v3.ctx, k) for k in range(3)] == [0, 1, 1]
        got = v3.verify_records(host, 0)
        assert (got == ver.verify_records(host, 0)).all()
        assert lib.hkv_debug_fail_device(v3.ctx, 0, 1) == 0
        with pytest.raises(HkvError) as e:
            v3.verify_records(host[: 1000 * 168], 1)
        assert e.value.rc == -4                            # HKV_E_HIP: no device left
        with pytest.raises(HkvError) as e:
            v3.verify_records(host[: 1000 * 168], 1)
        assert e.value.rc == -2                            # HKV_E_NODEV
        # the caller brings the devices back; an allocation failure (ADVICE
        # r03: HKV_E_OOM) fails the call but takes no device out of service
        for k in range(3):
            assert lib.hkv_device_reset_health(v3.ctx, k) == 0
        assert lib.hkv_debug_fail_device(v3.ctx, 1, 3) == 0   # HKV_FAIL_ALLOC
        with pytest.raises(HkvError) as e:
            v3.verify_records(host, 1)
        assert e.value.rc == -3                            # HKV_E_OOM
        assert [lib.hkv_device_healthy(v3.ctx, k) for k in range(3)] == [1, 1, 1]
        got = v3.verify_records(host, 1)
        assert (got == single).all()
        assert [lib.hkv_device_failures(v3.ctx, k) for k in range(3)] == [1, 1, 1]
    assert not single[bad].any() and single.sum() == n - bad.size


@pytest.mark.skipif(not os.environ.get("HKV_STRESS_RECORD_BATCHES"),
                    reason="stress run only (HKV_STRESS_RECORD_BATCHES=n)")
def test_record_byte_mutation_stress(torch, ver, coracle, openssl, secpfast):
    """Opt-in stress (profiles/r05p/): n batches of 262,144 generated records
    with 30 % of them damaged at one random byte (any of the 168: msg32, r,
    s, the key's length byte, prefix or coordinates, the padding) to a random
    value; the verdicts of both modes, at the full-grid launch shape, equal
    the C restatement's on every record, and (HKV_STRESS_OPENSSL=1) OpenSSL's
    behind the semantic adapter too, and the libsecp256k1-class restatement
    (oracle/secp_fast.c) always. HKV_STRESS_SEED0 starts at a later batch
    seed."""
    use_ossl = os.environ.get("HKV_STRESS_OPENSSL") == "1"
    n = 262144
    k0 = int(os.environ.get("HKV_STRESS_SEED0", "0"))
    for k in range(k0, k0 + int(os.environ["HKV_STRESS_RECORD_BATCHES"])):
        d = gen_device(torch, ver, n, seed=0x53545200 + k, unc=200)
        host = d.cpu().numpy().copy().reshape(-1, 168)
        rng = np.random.default_rng(0x5EED + k)
        hit = rng.random(n) < 0.3
        rows = np.nonzero(hit)[0]
        cols = rng.integers(0, 168, size=rows.size)
        host[rows, cols] = rng.integers(0, 256, size=rows.size, dtype=np.uint8)
        flat = host.reshape(-1)
        for mode in (0, 1):
            exp = oracle_batch(coracle, flat.tobytes(), mode, threads=host_threads())
            got = ver.verify_records(flat, mode)
            mism = np.nonzero(got != exp)[0]
            assert mism.size == 0, (k, mode, mism[:10], [int(c) for c in cols[np.isin(rows, mism[:10])]])
            mism = np.nonzero(got != fast_batch(secpfast, flat, mode, threads=host_threads()))[0]
            assert mism.size == 0, (k, mode, "secp_fast", mism[:10])
            if use_ossl:
                ossl = openssl_batch(openssl, flat.tobytes(), mode, threads=host_threads())
                mism = np.nonzero(got != ossl)[0]
                assert mism.size == 0, (k, mode, "openssl", mism[:10])
        print(f"record mutation stress: batch {k + 1}: {rows.size} damaged of {n}, accepts {int(got.sum())}"
              + (" (C restatement, secp_fast and OpenSSL)" if use_ossl else " (C restatement and secp_fast)"),
              flush=True)
