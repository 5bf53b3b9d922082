"""Batch header checks: headerHash + isValidPOW +
batch linkage, GPU (hkv_check_headers) against the CPU oracle
(oracle/header_oracle.py) and the header hashes the reference's own tests
assert (test/Haskoin/NodeSpec.hs:180-218, via tests/golden/ref_fixtures.json).
"""
import os
import json
import random

import numpy as np
import pytest

import header_oracle as ho
from conftest import GOLDEN

REGTEST = ho.POW_LIMIT["bchRegTest"]
MAINNET = ho.POW_LIMIT["btc"]


def fixture_headers():
    """The 15 bchRegTest fixture blocks' headers (heights 1..15)."""
    raw = open(os.path.join(GOLDEN, "ref_blocks.bin"), "rb").read()
    off, hdrs = 0, []
    while off < len(raw):
        hdrs.append(raw[off:off + 80])
        off += 80 + 1 + 4
        nin = raw[off]; off += 1
        for _ in range(nin):
            off += 36; sl = raw[off]; off += 1 + sl + 4
        nout = raw[off]; off += 1
        for _ in range(nout):
            off += 8; sl = raw[off]; off += 1 + sl
        off += 4
    return hdrs


def random_bits(rng: random.Random) -> int:
    """Adversarial and ordinary compact targets."""
    c = rng.randrange(8)
    if c == 0:
        return 0x207FFFFF                                   # regtest
    if c == 1:
        return 0x1D00FFFF                                   # mainnet genesis
    if c == 2:
        return (rng.randrange(0, 40) << 24) | rng.getrandbits(23)                   # any size, positive
    if c == 3:
        return (rng.randrange(0, 40) << 24) | 0x00800000 | rng.getrandbits(23)      # sign bit
    if c == 4:
        return (rng.choice([32, 33, 34, 35]) << 24) | rng.choice([0x1, 0xFF, 0x100, 0xFFFF, 0x10000, 0x7FFFFF])
    if c == 5:
        return (rng.randrange(0, 4) << 24) | rng.getrandbits(23)                    # size <= 3 shifts
    if c == 6:
        return ho.encode_compact(rng.getrandbits(rng.randrange(200, 256)))          # near the limit
    return (0x20 << 24) | rng.getrandbits(23)


def make_headers(n: int, seed: int, chain_frac: float = 0.5):
    """n headers: random fields and bits; a chain_frac share link to their
    predecessor (prev = hash of the header before)."""
    rng = random.Random(seed)
    out = []
    prev = bytes(32)
    for i in range(n):
        link = i > 0 and rng.random() < chain_frac
        p = ho.header_hash(out[-1]) if link else rng.randbytes(32)
        h = (rng.getrandbits(32).to_bytes(4, "little") + p + rng.randbytes(32) +
             rng.getrandbits(32).to_bytes(4, "little") + random_bits(rng).to_bytes(4, "little") +
             rng.getrandbits(32).to_bytes(4, "little"))
        out.append(h)
    return out


# ---------------------------------------------------------------- CPU -------

def test_oracle_fixture_chain():
    hdrs = fixture_headers()
    assert len(hdrs) == 15
    hashes, status = ho.check_headers(hdrs, REGTEST)
    fx = json.load(open(os.path.join(GOLDEN, "ref_fixtures.json")))["hashes"]
    disp = [h[::-1].hex() for h in hashes]
    assert disp[4:6] == fx["get_blocks"]          # NodeSpec.hs:180-183
    assert disp[14] == fx["best_h15"]             # :197-198
    assert disp[9] == fx["ancestor_h10"]          # :199-200
    assert disp[11:14] == fx["parents_of_h15"]    # :215-218
    assert all(s == ho.POW_OK | ho.LINK_OK for s in status)
    # the fixture chain fails the mainnet limit (0x207fffff target > powLimit)
    _, st2 = ho.check_headers(hdrs, MAINNET)
    assert all(s & ho.ABOVE_LIMIT and not s & ho.POW_OK for s in st2)


@pytest.mark.parametrize("bits,value,neg,over", [
    (0x00000000, 0, False, False),
    (0x00123456, 0, False, False),
    (0x01003456, 0, False, False),
    (0x02000056, 0, False, False),
    (0x01123456, 0x12, False, False),
    (0x02123456, 0x1234, False, False),
    (0x03123456, 0x123456, False, False),
    (0x04123456, 0x12345600, False, False),
    (0x04923456, 0x12345600, True, False),
    (0x05009234, 0x92340000, False, False),
    (0x01fedcba, 0x7e, True, False),
    (0x20123456, 0x123456 << 232, False, False),
    (0x1d00ffff, 0xffff << 208, False, False),
    (0x22000001, 1 << 248, False, False),
    (0x22000100, None, False, True),
    (0x21010000, None, False, True),
    (0x23000001, None, False, True),
    (0xff123456, None, False, True),
])
def test_decode_compact_known_answers(bits, value, neg, over):
    v, n, o = ho.decode_compact(bits)
    assert (n, o) == (neg, over)
    if value is not None:
        assert v == value


def test_encode_compact_round_trip():
    rng = random.Random(7)
    for _ in range(200):
        x = rng.getrandbits(rng.randrange(1, 256))
        v, neg, over = ho.decode_compact(ho.encode_compact(x))
        assert not neg and not over and v <= x and x - v < (1 << max(0, x.bit_length() - 15))


# ---------------------------------------------------------------- GPU -------

@pytest.fixture(scope="module")
def verifier():
    import torch
    import hkv
    # torch's HIP runtime first (as bench.py does), then the library's context
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    v = hkv.Verifier(hkv.VerifierConfig(device_ids=[0]))
    yield v
    v.close()


@pytest.mark.gpu
def test_gpu_fixture_chain(verifier):
    import hkv
    hdrs = fixture_headers()
    hashes, status = hkv.check_headers(verifier, hdrs, REGTEST)
    eh, es = ho.check_headers(hdrs, REGTEST)
    assert hashes == eh
    assert status.tolist() == es
    # header 0 against a tip: the right parent links, a wrong one does not
    _, st = hkv.check_headers(verifier, hdrs, REGTEST, prev_hash=hdrs[0][4:36])
    assert st[0] & ho.LINK_OK
    _, st = hkv.check_headers(verifier, hdrs, REGTEST, prev_hash=bytes(32))
    assert not st[0] & ho.LINK_OK and all(s & ho.LINK_OK for s in st[1:])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 255, 256, 257, 510, 511, 2000, 5003])
def test_gpu_random_headers_parity(verifier, n):
    import hkv
    hdrs = make_headers(n, seed=0x48445200 + n)
    prev = hdrs[0][4:36] if n % 2 else None
    for limit in (REGTEST, MAINNET):
        hashes, status = hkv.check_headers(verifier, hdrs, limit, prev_hash=prev)
        eh, es = ho.check_headers(hdrs, limit, prev_hash=prev)
        assert hashes == eh
        bad = [i for i in range(n) if status[i] != es[i]]
        assert not bad, [(i, hex(int.from_bytes(hdrs[i][72:76], "little")), status[i], es[i]) for i in bad[:5]]


@pytest.mark.gpu
def test_gpu_header_classes_all_seen(verifier):
    """The adversarial generator reaches every reject flag, so the parity
    test above covers each branch of isValidPOW."""
    import hkv
    hdrs = make_headers(4000, seed=11)
    seen = 0
    for limit in (REGTEST, MAINNET):
        _, status = hkv.check_headers(verifier, hdrs, limit)
        for s in status.tolist():
            seen |= s
    assert seen == 0x7F


@pytest.mark.gpu
def test_gpu_device_form_1m(verifier):
    """1M HBM-resident headers through the device entry point: hashes and
    flags of a random sample equal the oracle's; every header extends the one
    before it in a chained batch built on the host for a 4096-header slice."""
    import torch
    import hkv
    n = 1 << 20
    rng = np.random.default_rng(5)
    raw = rng.integers(0, 256, size=(n, 80), dtype=np.uint8)
    raw[:, 72:76] = np.frombuffer((0x207FFFFF).to_bytes(4, "little"), dtype=np.uint8)
    chain = make_headers(4096, seed=3, chain_frac=1.0)
    raw[:4096] = np.frombuffer(b"".join(chain), dtype=np.uint8).reshape(4096, 80)
    d = torch.from_numpy(raw.reshape(-1)).cuda()
    lim = torch.from_numpy(np.frombuffer(REGTEST.to_bytes(32, "little"), dtype=np.uint8).copy()).cuda()
    hashes = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    status = torch.zeros(n, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    hkv.check_headers_device(verifier, 0, d.data_ptr(), n, lim.data_ptr(), None, hashes.data_ptr(),
                             status.data_ptr(), s)
    torch.cuda.synchronize()
    hb = hashes.cpu().numpy().reshape(n, 32)
    st = status.cpu().numpy()
    assert all(st[1:4096] & ho.LINK_OK)
    idx = list(rng.choice(n, size=3000, replace=False)) + [0, 4095, 4096, n - 1]
    for i in idx:
        h = raw[i].tobytes()
        assert hb[i].tobytes() == ho.header_hash(h)
        exp = ho.pow_flags(h, REGTEST)
        if i == 0 or (i < 4096):
            exp |= ho.LINK_OK
        elif raw[i, 4:36].tobytes() == hb[i - 1].tobytes():
            exp |= ho.LINK_OK
        assert st[i] == exp, i
    # regtest target ~2^255: about half of random hashes pass
    frac = float((st & ho.POW_OK).astype(bool).mean())
    assert 0.45 < frac < 0.55
