"""The Verify actor on the MI355X: hkv/actor.py — the
mirror of withVerifyActor in haskell/Haskoin/Node/Verify.hs — coalesces
single-tx mempool events into few hkv_verify_std_inputs calls, and a call
whose multisig tail gives up (the HKV_FAIL_TAIL hook) is re-submitted (or
handed to the caller's CPU path) instead of raising: every verdict equals the
oracle's. Actor idiom: /root/reference/src/Haskoin/Node/Chain.hs:277-307;
events: /root/reference/src/Haskoin/Node.hs:151-174."""
import random
from collections import defaultdict

import pytest

import sighash_oracle as sh
from conftest import host_threads, oracle_batch

pytestmark = pytest.mark.gpu


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


def _events(txs, inputs):
    """One event per tx: (key, tx bytes, [(input index, prevout script, value)])."""
    per = defaultdict(list)
    for (t, i, spk, val) in inputs:
        per[t].append((i, spk, val))
    return [(f"tx{t}", txs[t], per[t]) for t in range(len(txs))]


def _outcomes(events, verdicts):
    from hkv.actor import TxRejected, TxVerified
    out = []
    for (key, _, ins), vs in zip(events, verdicts):
        bad = tuple(i for (i, _, _), v in zip(ins, vs) if not v)
        out.append(TxRejected(key, bad) if bad else TxVerified(key))
    return out


def _run(ver, events, **cfg):
    from hkv.actor import VerifyActor, VerifyActorConfig
    out = []
    a = VerifyActor(ver, out.append, VerifyActorConfig(**cfg))
    for e in events:
        a.verify_tx(*e)
    a.start()
    a.stop()
    return a, out


def test_mempool_events_coalesce_into_few_calls(torch, ver, coracle):
    """5,000 single-tx events (P2PKH + P2WPKH, 2-5 inputs each, one input in
    20 txs given a wrong prevout: a P2WPKH value off by one or a P2PKH hash
    of another key) -> at most ceil(inputs / 16,384) + 2 GPU calls, every
    outcome equal to the oracle's (every input's record re-derived by
    oracle/sighash_oracle.py, verdicts by the C restatement)."""
    from hkv import blockgen
    txs, inputs = blockgen.make_block(ver, torch, n_tx=5000, seed=0x484B5641, inputs_per_tx=(2, 3, 4, 5))
    rng = random.Random(0x484B5641)
    inputs = list(inputs)
    for k, (t, i, spk, val) in enumerate(inputs):
        if i == 0 and t % 20 == 7:
            inputs[k] = (t, i, spk, val + 1) if spk[:2] == b"\x00\x14" else (t, i, spk[:3] + rng.randbytes(20) + spk[23:],
                                                                             val)
    events = _events(txs, inputs)
    n_in = len(inputs)
    assert len(events) == 5000 and 15000 < n_in < 20000
    parsed = [sh.tx_parse(t) for t in txs]
    recs = b"".join(sh.std_input_record(parsed[t], i, p, v) for (t, i, p, v) in inputs)
    want_flat = oracle_batch(coracle, recs, 1, threads=host_threads()).tolist()
    pos = {(t, i): k for k, (t, i, _, _) in enumerate(inputs)}
    want = [[want_flat[pos[(t, i)]] for (i, _, _) in ins] for t, (_, _, ins) in enumerate(events)]
    assert 200 <= sum(not v for v in want_flat) <= 300
    a, out = _run(ver, events, max_inputs=16384, max_wait_s=0.5)
    assert out == _outcomes(events, want)
    assert a.stats.gpu_failures == 0 and a.stats.fallback_calls == 0
    assert a.stats.gpu_calls <= -(-n_in // 16384) + 2
    assert sum(a.stats.batch_inputs) == n_in and max(a.stats.batch_inputs) <= 16384


def _ms_events():
    from test_gpu_sighash import _ms_block
    rng = random.Random(0x484B5642)
    raw, jobs, labels = _ms_block(rng, None)
    return raw, jobs, _events(raw, jobs)


def _ms_want(coracle, raw, jobs, events):
    from test_gpu_sighash import _ms_oracle
    flat = _ms_oracle(coracle, raw, jobs, None)
    pos = {(t, i): k for k, (t, i, _, _) in enumerate(jobs)}
    return [[flat[pos[(t, i)]] for (i, _, _) in ins] for t, (_, _, ins) in enumerate(events)], flat


def test_tail_fault_is_resubmitted_not_raised(torch, ver, coracle):
    """A mempool batch holding multisig inputs whose tail gives up (forced):
    the actor re-submits it once and publishes the oracle's outcomes."""
    from hkv.lib import HKV_FAIL_TAIL
    raw, jobs, events = _ms_events()
    want, flat = _ms_want(coracle, raw, jobs, events)
    assert sum(flat) > 40
    assert ver.lib.hkv_debug_fail_device(ver.ctx, 0, HKV_FAIL_TAIL) == 0
    a, out = _run(ver, events, max_wait_s=0.5, retries=1)
    assert out == _outcomes(events, want)
    assert a.stats.gpu_calls == 2 and a.stats.gpu_failures == 1 and a.stats.fallback_calls == 0
    assert "hkv_verify_std_inputs" in a.stats.errors[0]
    ver.device_fault(0)  # (clear the latch the forced fault set)


def test_tail_fault_goes_to_the_callers_cpu_path(torch, ver, coracle):
    """retries = 0: the faulted batch goes to the caller's CPU path (in the
    Haskell actor haskoin-core's verifyStdInput; here the test's checker
    stands in for it) with exactly that batch, and the outcomes equal the
    oracle's; the next batch is back on the GPU."""
    from hkv.lib import HKV_FAIL_TAIL
    from test_gpu_sighash import _ms_oracle
    raw, jobs, events = _ms_events()
    want, _ = _ms_want(coracle, raw, jobs, events)
    seen = []

    def cpu_path(txs, inputs, forkid):
        seen.append(len(inputs))
        return _ms_oracle(coracle, list(txs), list(inputs), forkid)

    assert ver.lib.hkv_debug_fail_device(ver.ctx, 0, HKV_FAIL_TAIL) == 0
    a, out = _run(ver, events, max_wait_s=0.5, retries=0, fallback=cpu_path)
    assert out == _outcomes(events, want)
    assert a.stats.gpu_calls == 1 and a.stats.gpu_failures == 1 and a.stats.fallback_calls == 1
    assert seen == [len(jobs)]
    ver.device_fault(0)
    a, out = _run(ver, events, max_wait_s=0.5, retries=0, fallback=cpu_path)
    assert out == _outcomes(events, want) and a.stats.fallback_calls == 0 and a.stats.gpu_calls == 1
