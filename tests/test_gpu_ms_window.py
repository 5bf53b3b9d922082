"""The multisig tail's record windows: the candidate and
key-check records of a chunk run in rounds through windows capped at
~512 MiB instead of buffers sized by the 16-of-16 bound (3.35 GB per
131,072-input chunk). Verdicts must equal the oracle's whatever the window
(forced small with hkv_debug_ms_window, so that records straddle rounds),
a 131,072-input all-multisig chunk must equal the oracle, and a chunk holds
at most the budget whether it has multisig inputs or not. Data source:
blocks from getBlocks, /root/reference/src/Haskoin/Node/Peer.hs:309-324."""
import ctypes
import random

import pytest

import secp256k1_oracle as o
import sighash_oracle as sh
from conftest import host_threads, oracle_batch

pytestmark = pytest.mark.gpu

BUDGET = 512 << 20


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need the MI355X"
    return t


@pytest.fixture(scope="module")
def ver(torch):
    import hkv
    v = hkv.Verifier(hkv.VerifierConfig(device_ids=[0], flags=1))
    yield v
    v.close()


def _window(ver, cand, keys):
    assert ver.lib.hkv_debug_ms_window(ver.ctx, 0, cand, keys) == 0


def _scratch(ver):
    b = ctypes.c_size_t()
    assert ver.lib.hkv_debug_ms_scratch(ver.ctx, 0, ctypes.byref(b)) == 0
    return b.value


def batched_oracle(coracle, raw_txs, jobs, forkid=None):
    """The oracle's verifyStdInput over every job (oracle/sighash_oracle.py
    verify_std_input: countMulSig over candidate verdicts), with ONE C-oracle
    call for every candidate record of the batch: a first pass collects the
    records (placeholder verdicts), a second replays each walk on the real
    ones. Key parses are memoised (keys repeat from a pool)."""
    parsed = [sh.tx_parse(t) for t in raw_txs]
    memo = {}

    def key_ok(k):
        if k not in memo:
            memo[k] = o.pubkey_parse(k) is not None
        return memo[k]

    recs, spans = [], []

    def collect(rs):
        spans.append((len(recs), len(rs)))
        recs.extend(rs)
        return [True] * len(rs)

    for (t, i, p, v) in jobs:
        n0 = len(spans)
        sh.verify_std_input(parsed[t], i, p, v, forkid, collect, key_ok)
        if len(spans) == n0:
            spans.append((len(recs), 0))
    flat = oracle_batch(coracle, b"".join(recs), 1, threads=host_threads()).tolist() if recs else []
    out = []
    for k, (t, i, p, v) in enumerate(jobs):
        a, n = spans[k]
        out.append(sh.verify_std_input(parsed[t], i, p, v, forkid, lambda rs: flat[a:a + n], key_ok))
    return out


@pytest.mark.parametrize("cand,keys", [(64, 64), (4096, 256), (0, 0)])
def test_forced_windows_equal_oracle(torch, ver, coracle, cand, keys):
    """Every multisig case of tests/txgen.py (all wraps and variants) beside
    signed single-signature txs, through the block kernel and the host form,
    with windows of 64 / 4,096 candidate records (tens of rounds) and the
    default: verdicts equal the oracle's each time."""
    import hkv
    from test_gpu_sighash import _device_verify_std, _ms_block
    rng = random.Random(0x57 + cand)
    raw, jobs, labels = _ms_block(rng, None)
    want = batched_oracle(coracle, raw, jobs)
    _window(ver, cand, keys)
    try:
        got = _device_verify_std(torch, ver, raw, jobs, None)
        bad = [(labels[k], got[k], want[k]) for k in range(len(jobs)) if got[k] != want[k]]
        assert not bad, bad[:10]
        assert hkv.verify_std_inputs(ver, raw, jobs) == want
    finally:
        _window(ver, 0, 0)
    assert sum(g for g, lb in zip(want, labels) if lb != "single") > 40
    assert ver.device_fault(0) == 0


@pytest.mark.timeout(900)
def test_full_chunk_all_multisig_equals_oracle(torch, ver, coracle):
    """131,072 multisig inputs (one chunk: 1-of-1 .. 3-of-3, every wrap, 8 %
    damaged), device-signed: verdicts equal the oracle's at the default
    windows and with windows forced to 65,536 candidate / 16,384 key records
    (several rounds); the record windows stay within the ~512 MiB budget."""
    import hkv
    from hkv import blockgen
    txs, inputs = blockgen.make_multisig_block(ver, torch, n_tx=131072)
    assert len(inputs) == 131072
    want = batched_oracle(coracle, txs, inputs)
    assert 0.85 * len(want) < sum(want) < 0.97 * len(want)
    got = hkv.verify_std_inputs(ver, txs, inputs)
    assert got == want
    assert _scratch(ver) <= BUDGET
    _window(ver, 65536, 16384)
    try:
        assert hkv.verify_std_inputs(ver, txs, inputs) == want
    finally:
        _window(ver, 0, 0)
    assert ver.device_fault(0) == 0


def test_multisig_free_chunk_within_budget(torch):
    """A fresh context given a 75,000-tx single-signature batch (> one
    131,072-input chunk) holds at most the budget of multisig records (the
    16-of-16 bound would be 3.35 GB)."""
    import hkv
    from hkv import blockgen
    with hkv.Verifier(hkv.VerifierConfig(device_ids=[0], flags=1)) as v:
        txs, inputs = blockgen.make_block(v, torch, n_tx=75000, seed=0x484B5644)
        assert len(inputs) > 131072
        assert all(hkv.verify_std_inputs(v, txs, inputs))
        b = ctypes.c_size_t()
        assert v.lib.hkv_debug_ms_scratch(v.ctx, 0, ctypes.byref(b)) == 0
        assert 0 < b.value <= BUDGET


@pytest.mark.timeout(900)
def test_two_chunks_with_multisig_on_both_sides(torch, ver, coracle):
    """A batch past one 131,072-input chunk with multisig inputs in both
    chunks (6,000 multisig inputs, 126,000 single-signature inputs, 6,000
    more multisig inputs: the chunk boundary falls among the single-signature
    inputs, so each chunk holds multisig inputs and the second chunk's jobs
    start mid-batch): each chunk runs its own scan, windows and tail; verdicts
    of the host form and of the device form with a status word equal the
    oracle's, with no fault."""
    import hkv
    from hkv import blockgen
    from test_gpu_sighash import _device_verify_std
    mt1, mi1 = blockgen.make_multisig_block(ver, torch, n_tx=6000, seed=0x484B5647)
    st_, si = blockgen.make_block(ver, torch, n_tx=76000, seed=0x484B5648, inputs_per_tx=(1, 2, 2, 2))
    mt2, mi2 = blockgen.make_multisig_block(ver, torch, n_tx=6000, seed=0x484B5649)
    txs = mt1 + st_ + mt2
    o1, o2 = len(mt1), len(mt1) + len(st_)
    si = si[:126000]
    inputs = list(mi1) + [(t + o1, i, p, v) for (t, i, p, v) in si] + [(t + o2, i, p, v) for (t, i, p, v) in mi2]
    assert len(si) == 126000 and len(inputs) == 138000 and len(mi1) + len(si) > 131072 > len(mi1)
    want = batched_oracle(coracle, txs, inputs)
    assert 0 < sum(not w for w in want) < 2000
    assert hkv.verify_std_inputs(ver, txs, inputs) == want
    got, st = _device_verify_std(torch, ver, txs, inputs, None, status=True)
    assert st == 0 and got == want
    assert ver.device_fault(0) == 0


@pytest.mark.timeout(1200)
def test_past_one_grid_full_grid_chunks(torch, ver, coracle):
    """A batch past one resident grid (262,144 inputs) runs in chunks of up
    to 2^20 inputs through the full-grid instance (extraction, then the record
    verify at 4 waves per SIMD) instead of half-grid chunks: ~290,000 inputs,
    multisig inputs at both ends, in one chunk through the host form and the
    device form with a status word; and with HKV_STD_CHUNK=196608 (a fresh
    context) as a full-grid chunk of 196,608 inputs followed by a half-grid
    one — every verdict equal to the oracle's, no fault."""
    import os
    import hkv
    from hkv import blockgen
    from test_gpu_sighash import _device_verify_std
    mt1, mi1 = blockgen.make_multisig_block(ver, torch, n_tx=3000, seed=0x484B564A)
    st_, si = blockgen.make_block(ver, torch, n_tx=163000, seed=0x484B564B, inputs_per_tx=(1, 2, 2, 2))
    mt2, mi2 = blockgen.make_multisig_block(ver, torch, n_tx=3000, seed=0x484B564C)
    txs = mt1 + st_ + mt2
    o1, o2 = len(mt1), len(mt1) + len(st_)
    inputs = list(mi1) + [(t + o1, i, p, v) for (t, i, p, v) in si] + [(t + o2, i, p, v) for (t, i, p, v) in mi2]
    assert len(inputs) > 262144 + 20000
    want = batched_oracle(coracle, txs, inputs)
    assert 0 < sum(not w for w in want) < 1000
    assert hkv.verify_std_inputs(ver, txs, inputs) == want
    got, st = _device_verify_std(torch, ver, txs, inputs, None, status=True)
    assert st == 0 and got == want
    assert ver.device_fault(0) == 0
    os.environ["HKV_STD_CHUNK"] = "196608"
    try:
        with hkv.Verifier(hkv.VerifierConfig(device_ids=[0], flags=1)) as v2:
            got, st = _device_verify_std(torch, v2, txs, inputs, None, status=True)
            assert st == 0 and got == want
            assert v2.device_fault(0) == 0
    finally:
        del os.environ["HKV_STD_CHUNK"]
