"""GPU parity tests (MI355X): the HIP path through the C ABI against the
oracle — bit-exact verdicts, both modes, golden KATs, random and adversarial
batches, field/scalar known answers, determinism, the 1M-record size."""
import ctypes
import random

import numpy as np
import pytest

import secp256k1_oracle as o
from conftest import oracle_batch

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


def adversarial(host: np.ndarray, seed: int) -> np.ndarray:
    """Mutate ~30% of valid records into SURVEY §8(c) invalid classes (config 4)."""
    rng = np.random.default_rng(seed)
    a = host.reshape(-1, 168).copy()
    n = a.shape[0]
    cls = rng.integers(0, 20, size=n)  # 0..5 -> mutated (30%)
    idx = np.nonzero(cls == 0)[0]; a[idx, rng.integers(0, 32, len(idx))] ^= 1            # msg bit
    idx = np.nonzero(cls == 1)[0]; a[idx, 32:64] = 0                                      # r = 0
    idx = np.nonzero(cls == 2)[0]; a[idx, 64:96] = 0xFF                                   # s >= n
    idx = np.nonzero(cls == 3)[0]; a[idx, 97] ^= 0x04                                     # bad prefix
    idx = np.nonzero(cls == 4)[0]; a[idx, 98:130] = 0xFF                                  # x >= p
    idx = np.nonzero(cls == 5)[0]                                                         # high-S
    for i in idx:
        s = int.from_bytes(a[i, 64:96].tobytes(), "big")
        a[i, 64:96] = np.frombuffer((o.N - s).to_bytes(32, "big"), dtype=np.uint8)
    return a.reshape(-1)


def test_generated_valid_batch_all_accept_and_oracle_agrees(torch, ver, coracle):
    n = 65536 + 17
    d = gen_device(torch, ver, n, seed=0x484B5632)
    host = d.cpu().numpy()
    got = ver.verify_records(host, 0)
    assert got.all(), int((~got).sum())
    # the generator's records are valid per the independent oracle (sample)
    exp = oracle_batch(coracle, host[: 4096 * 168].tobytes(), 0, threads=16)
    assert exp.all()


def test_adversarial_batch_vs_oracle(torch, ver, coracle):
    n = 131072
    d = gen_device(torch, ver, n, seed=0x484B5634, unc=100)
    adv = adversarial(d.cpu().numpy(), 11)
    for mode in (0, 1):
        exp = oracle_batch(coracle, adv.tobytes(), mode, threads=16)
        got = ver.verify_records(adv, mode)
        mism = np.nonzero(got != exp)[0]
        assert mism.size == 0, (mode, mism[:20])
        assert 0.6 < exp.mean() < 0.8


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


def test_config4_adversarial_1m_both_modes(torch, ver, coracle):
    """BASELINE configs[3]: 1,048,576 records, 30% invalid over the §8(c)
    classes, exact reject parity in both modes against the construction labels
    (hkv/adversarial.py, pinned per class by test_adversarial_labels.py) and a
    32k slice against the C oracle."""
    from hkv import adversarial
    n = 1 << 20
    d = gen_device(torch, ver, n, seed=0x484B5634)
    adv, lab_lib, lab_hask, cls = adversarial.mutate(d.cpu().numpy(), seed=0x484B5634)
    assert 0.29 < (cls >= 0).mean() < 0.31
    d.copy_(torch.from_numpy(adv))
    for mode, lab in ((0, lab_lib), (1, lab_hask)):
        got = adversarial.unpack_bits(verify_dev_bits(torch, ver, d, n, mode), n)
        mism = np.nonzero(got != lab)[0]
        assert mism.size == 0, (mode, mism[:10], cls[mism[:10]])
        sl = slice(500_000 * 168, (500_000 + 32768) * 168)
        exp = oracle_batch(coracle, adv[sl].tobytes(), mode, threads=16)
        assert (got[500_000:500_000 + 32768] == exp).all()


def test_config5_ibd_16m_sharded_bitmap(torch, ver):
    """BASELINE configs[4] shape on one GPU: 16,777,216 records (config-2
    distribution, 5% invalid), verified as the 8 contiguous shards of the
    8-GPU run (hkv/shard.py) and assembled as the all-gather does; the bitmap
    equals the single-launch bitmap and the construction labels bit for bit."""
    from hkv import adversarial
    from hkv.shard import assemble_bitmap, shard_bounds
    n, world = 1 << 24, 8
    d = gen_device(torch, ver, n, seed=0x484B5635)
    adv, lab, _, _ = adversarial.mutate(d.cpu().numpy(), seed=0x484B5635, invalid_frac=0.05)
    d.copy_(torch.from_numpy(adv))
    del adv
    whole = verify_dev_bits(torch, ver, d, n, 0)[: (n + 31) // 32]
    wpr = (n // world + 63) // 64 * 2 + 2
    gathered = np.zeros(world * wpr, dtype=np.uint32)
    for r in range(world):
        lo, hi = shard_bounds(n, r, world)
        w = verify_dev_bits(torch, ver, d, hi - lo, 0, offset=lo)
        gathered[r * wpr: r * wpr + w.size] = w
    full = assemble_bitmap(n, world, gathered, wpr)
    assert (full == whole).all()
    got = adversarial.unpack_bits(full, n)
    assert (got == lab).all(), np.nonzero(got != lab)[0][:10]


def test_split_lane_ecmult_matches_full_grid(torch, ver, coracle):
    """Small batches run two lanes per signature (hkv_ecmult_kernel<true>,
    chosen when the padded batch fills at most an eighth of the resident
    grid, 32,768 signatures on an MI355X);
    large ones one lane (<false>). The same adversarial records verified in
    both launch shapes give identical verdicts, equal to the C oracle on a
    slice, in both modes."""
    from hkv import adversarial
    n_small, n_big = 1 << 15, (1 << 15) + 257          # n_pad 32,768 (split) / 33,024 (full)
    d = gen_device(torch, ver, n_big, seed=0x53504C54)
    adv, lab_lib, lab_hask, _ = adversarial.mutate(d.cpu().numpy(), seed=0x53504C54)
    d.copy_(torch.from_numpy(adv))
    for mode, lab in ((0, lab_lib), (1, lab_hask)):
        small = adversarial.unpack_bits(verify_dev_bits(torch, ver, d, n_small, mode), n_small)
        big = adversarial.unpack_bits(verify_dev_bits(torch, ver, d, n_big, mode), n_big)
        assert (small == big[:n_small]).all()
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
