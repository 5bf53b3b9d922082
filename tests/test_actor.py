"""The Verify actor's batching and error policy on the CPU (hkv/actor.py, the
mirror of withVerifyActor in haskell/Haskoin/Node/Verify.hs). The GPU call is
replaced by a recording stub here (its verdict of input (tx, i) is a fixed
function of the tx bytes and i); tests/test_gpu_actor.py runs the same actor
through libhkv on the MI355X against the oracle."""
import time

import pytest

import hkv.actor as actor
from hkv.actor import (BlockRejected, BlockVerified, TxRejected, TxVerified, VerifyActor, VerifyActorConfig,
                       VerifyFailed)
from hkv.lib import HkvError


def verdict(tx: bytes, i: int) -> bool:
    return (tx[0] + 3 * i) % 5 != 0


class StubGPU:
    """verify_std_inputs stand-in: records every call; fails the calls whose
    ordinal is in `fail` with HKV_E_INTERNAL (-5)."""

    def __init__(self, fail=()):
        self.calls, self.fail = [], set(fail)

    def __call__(self, v, txs, inputs, forkid):
        self.calls.append((len(txs), len(inputs), forkid))
        if len(self.calls) in self.fail:
            raise HkvError(-5, "hkv_verify_std_inputs")
        return [verdict(txs[t], i) for (t, i, _, _) in inputs]


def tx_events(n, rng_seed=7, max_in=4):
    import random
    rng = random.Random(rng_seed)
    out = []
    for k in range(n):
        tx = bytes([rng.randrange(256)]) + k.to_bytes(4, "little")
        out.append((f"tx{k}", tx, [(i, b"\x51", 1000 + i) for i in range(rng.randrange(1, max_in + 1))]))
    return out


def expected(events):
    res = []
    for key, tx, ins in events:
        bad = tuple(i for (i, _, _) in ins if not verdict(tx, i))
        res.append(TxRejected(key, bad) if bad else TxVerified(key))
    return res


def run(events, cfg, stub, monkeypatch, blocks=()):
    monkeypatch.setattr(actor, "verify_std_inputs", stub)
    out = []
    a = VerifyActor(None, out.append, cfg)
    for e in events:
        if e[0].startswith("blk"):
            a.verify_block(*e)
        else:
            a.verify_tx(*e)
    a.start()
    a.stop()
    return a, out


def test_coalesces_mempool_txs_into_few_calls(monkeypatch):
    ev = tx_events(5000)
    n_in = sum(len(x[2]) for x in ev)
    stub = StubGPU()
    a, out = run(ev, VerifyActorConfig(max_inputs=4096, max_wait_s=1.0), stub, monkeypatch)
    assert out == expected(ev)
    assert len(stub.calls) <= -(-n_in // 4096) + 1
    assert all(n <= 4096 for (_, n, _) in stub.calls) and sum(n for (_, n, _) in stub.calls) == n_in
    assert a.stats.gpu_calls == len(stub.calls) and a.stats.gpu_failures == 0


def test_wait_bound_flushes_a_partial_batch(monkeypatch):
    """A lone tx is verified after max_wait_s, not held for more input."""
    stub = StubGPU()
    monkeypatch.setattr(actor, "verify_std_inputs", stub)
    out = []
    a = VerifyActor(None, out.append, VerifyActorConfig(max_inputs=10**6, max_wait_s=0.05)).start()
    a.verify_tx("a", b"\x01abc", [(0, b"\x51", 1)])
    t0 = time.time()
    while not out and time.time() - t0 < 10:
        time.sleep(0.005)
    assert out == [TxVerified("a")] and stub.calls == [(1, 1, None)]
    a.stop()


def test_blocks_keep_mailbox_order(monkeypatch):
    ev = tx_events(30)
    blk = ("blk0", [b"\x05\x00", b"\x07\x01"], [(0, 0, b"\x51", 5), (1, 0, b"\x51", 6), (1, 1, b"\x51", 6)])
    seq = ev[:10] + [blk] + ev[10:]
    stub = StubGPU()
    a, out = run(seq, VerifyActorConfig(max_inputs=10**6, max_wait_s=1.0), stub, monkeypatch)
    want_blk = BlockRejected("blk0", ((0, 0), (1, 1)))  # (5 + 0) % 5 == 0 and (7 + 3) % 5 == 0
    assert out == expected(ev[:10]) + [want_blk] + expected(ev[10:])
    assert len(stub.calls) == 3  # txs before the block, the block, txs after


def test_oversized_tx_is_its_own_batch(monkeypatch):
    ev = tx_events(6, max_in=2)
    big = ("big", b"\x09big", [(i, b"\x51", 1) for i in range(50)])
    stub = StubGPU()
    a, out = run(ev[:3] + [big] + ev[3:], VerifyActorConfig(max_inputs=20, max_wait_s=1.0), stub, monkeypatch)
    assert out == expected(ev[:3] + [big] + ev[3:])
    assert [n for (_, n, _) in stub.calls].count(50) == 1


def test_failed_call_is_resubmitted(monkeypatch):
    ev = tx_events(200)
    stub = StubGPU(fail={1})
    a, out = run(ev, VerifyActorConfig(max_inputs=10**6, max_wait_s=1.0, retries=1), stub, monkeypatch)
    assert out == expected(ev)
    assert a.stats.gpu_calls == 2 and a.stats.gpu_failures == 1 and a.stats.fallback_calls == 0


def test_fallback_after_retries(monkeypatch):
    ev = tx_events(50)
    seen = []

    def fallback(txs, inputs, forkid):
        seen.append(len(inputs))
        return [verdict(txs[t], i) for (t, i, _, _) in inputs]

    stub = StubGPU(fail={1, 2})
    a, out = run(ev, VerifyActorConfig(max_inputs=10**6, max_wait_s=1.0, retries=1, fallback=fallback), stub,
                 monkeypatch)
    assert out == expected(ev)
    assert a.stats.gpu_calls == 2 and a.stats.fallback_calls == 1 and seen == [sum(len(x[2]) for x in ev)]


def test_no_fallback_publishes_failures_and_keeps_running(monkeypatch):
    ev = tx_events(20)
    stub = StubGPU(fail={1})
    a, out = run(ev[:10] + [("blk1", [b"\x01"], [(0, 0, b"\x51", 1)])] + ev[10:],
                 VerifyActorConfig(max_inputs=10**6, max_wait_s=1.0, retries=0), stub, monkeypatch)
    assert all(isinstance(x, VerifyFailed) for x in out[:10])
    assert out[10] == BlockVerified("blk1") and out[11:] == expected(ev[10:])


def test_bad_config_rejected():
    with pytest.raises(ValueError):
        VerifyActor(None, print, VerifyActorConfig(max_inputs=0))


def test_failing_fallback_publishes_failures_and_keeps_running(monkeypatch):
    """A fallback that raises (or answers the wrong number of verdicts) leaves
    the batch unverified: VerifyFailed for its messages, and the actor goes on
    with the next ones."""
    ev = tx_events(12)
    calls = []

    def fallback(txs, inputs, forkid):
        calls.append(len(inputs))
        if len(calls) == 1:
            raise OSError("cpu path down")
        return [True]  # wrong length
    stub = StubGPU(fail={1, 2})
    blk = ("blk2", [b"\x01"], [(0, 0, b"\x51", 1), (0, 1, b"\x51", 1)])
    a, out = run(ev[:6] + [blk] + ev[6:], VerifyActorConfig(max_inputs=10**6, max_wait_s=1.0, retries=0,
                                                          fallback=fallback), stub, monkeypatch)
    assert all(isinstance(x, VerifyFailed) for x in out[:7]) and "cpu path down" in out[0].error
    assert "verdicts" in out[6].error
    assert out[7:] == expected(ev[6:]) and a.stats.fallback_calls == 2


def test_posting_to_a_crashed_actor_raises(monkeypatch):
    monkeypatch.setattr(actor, "verify_std_inputs", StubGPU())

    def publish(_):
        raise KeyError("subscriber bug")
    a = VerifyActor(None, publish, VerifyActorConfig(max_wait_s=0.01)).start()
    a.verify_tx("a", b"\x01abc", [(0, b"\x51", 1)])
    a._thread.join(10)
    with pytest.raises(RuntimeError):
        a.verify_tx("b", b"\x02abc", [(0, b"\x51", 1)])
    with pytest.raises(KeyError):
        a.stop()
