"""verifyStdInput readings taken without haskoin-core source (DESIGN.md §2,
"Multisig" / "Wrapped templates" / "Deliberate limits"): one named case per
reading, stating the reading the oracle and the kernels take and the
alternative a maintainer with haskoin-core-1.1.0 [dep, /root/reference/
stack.yaml:10] should check it against. Each case is built so that the two
readings give DIFFERENT verdicts, so the test pins which one is implemented:

  reading                                   chosen   alternative
  empty witness item in P2WSH multisig      valid    invalid (not TxSignatureEmpty:
    is TxSignatureEmpty (consumes a key)              the witness decode fails)
  P2PK key as a non-canonical push          invalid  valid (decodeOutput accepts it and
    (4c 21 <33> ac)                                   encodeOutput's canonical script is signed)
  multisig key as a non-canonical push      invalid  valid (same re-encoding)
  countMulSig == m (not >= m)               invalid  valid (an extra valid signature counts)
  an undecodable item past the n-th         invalid  valid (items beyond n are ignored)

The CPU tests check the oracle (oracle/sighash_oracle.py); the GPU tests run
the same inputs through hkv_verify_std_inputs (host form) and
hkv_verify_std_inputs_device (the fused small-batch kernel) and require the
chosen verdict from both. Parity unpinned: no reference fixture holds any of
these spends."""
import hashlib
import random

import pytest

import secp256k1_oracle as o
import sighash_oracle as sh
import txgen

ALT = {"empty_witness_item": False, "p2pk_pushdata1": True, "multisig_pushdata1_key": True,
       "count_above_m": True, "undecodable_past_n": True}
CHOSEN = {k: not v for k, v in ALT.items()}


def _keys(rng, n):
    return [txgen.Key(rng.randrange(1, o.N)) for _ in range(n)]


def _sig(tx, code, value, i, key, rng, segwit=False, shb=0x01):
    msg = sh.sighash_forkid(tx, code, value, i, shb) if segwit else sh.sighash_legacy(tx, code, value, i, shb)
    r, s = txgen.sign(msg, key.d, rng.randrange(1, o.N))
    return sh.der_encode(r, s) + bytes([shb])


def reading_cases():
    """(name, txs, jobs) per reading; jobs = [(tx index, input, prevout script, value)]."""
    rng = random.Random(0x52454144)
    out = []
    # 1. P2WSH 2-of-3: witness [dummy, empty, sig(k1), sig(k2), ws] — the empty
    #    item consumes key 0, the signatures match keys 1 and 2
    ks = _keys(rng, 3)
    ws = txgen.multisig_script(2, [k.pub for k in ks])
    prog = b"\x00\x20" + hashlib.sha256(ws).digest()
    tx = txgen._ms_tx(rng)
    value = rng.randrange(1, 2**40)
    tx.witness[0] = [b"", b"", _sig(tx, ws, value, 0, ks[1], rng, True), _sig(tx, ws, value, 0, ks[2], rng, True), ws]
    tx.inputs[0].script = b""
    out.append(("empty_witness_item", [tx], [(0, 0, prog, value)]))
    # 2. P2PK with the key pushed by PUSHDATA1, signed over the canonical script
    k = _keys(rng, 1)[0]
    canon = txgen.push(k.pub) + b"\xac"
    noncanon = b"\x4c" + bytes([len(k.pub)]) + k.pub + b"\xac"
    tx = txgen._ms_tx(rng)
    value = rng.randrange(1, 2**40)
    tx.inputs[0].script = txgen.push(_sig(tx, canon, value, 0, k, rng))
    out.append(("p2pk_pushdata1", [tx], [(0, 0, noncanon, value)]))
    # 3. bare 1-of-2 with key 0 pushed by PUSHDATA1, signed over the canonical script
    ks = _keys(rng, 2)
    canon = txgen.multisig_script(1, [k.pub for k in ks])
    noncanon = b"\x51\x4c" + bytes([len(ks[0].pub)]) + ks[0].pub + txgen.push(ks[1].pub) + b"\x52\xae"
    tx = txgen._ms_tx(rng)
    value = rng.randrange(1, 2**40)
    tx.inputs[0].script = b"\x00" + txgen.push(_sig(tx, canon, value, 0, ks[0], rng))
    out.append(("multisig_pushdata1_key", [tx], [(0, 0, noncanon, value)]))
    # 4. bare 1-of-2 with two valid signatures (keys 0 and 1): count 2 != 1
    ks = _keys(rng, 2)
    script = txgen.multisig_script(1, [k.pub for k in ks])
    tx = txgen._ms_tx(rng)
    value = rng.randrange(1, 2**40)
    tx.inputs[0].script = b"\x00" + txgen.push(_sig(tx, script, value, 0, ks[0], rng)) + \
        txgen.push(_sig(tx, script, value, 0, ks[1], rng))
    out.append(("count_above_m", [tx], [(0, 0, script, value)]))
    # 5. bare 1-of-1: the valid signature, then an undecodable item (item 2 > n = 1)
    ks = _keys(rng, 1)
    script = txgen.multisig_script(1, [ks[0].pub])
    tx = txgen._ms_tx(rng)
    value = rng.randrange(1, 2**40)
    tx.inputs[0].script = b"\x00" + txgen.push(_sig(tx, script, value, 0, ks[0], rng)) + \
        txgen.push(b"\x30\x02\x01\x01\x01")
    out.append(("undecodable_past_n", [tx], [(0, 0, script, value)]))
    return out


def _controls():
    """The same spends with the contested detail removed verify under both
    readings (so a False above is the reading, not a broken construction)."""
    rng = random.Random(0x434F4E54)
    out = []
    k = _keys(rng, 1)[0]
    canon = txgen.push(k.pub) + b"\xac"
    tx = txgen._ms_tx(rng)
    value = rng.randrange(1, 2**40)
    tx.inputs[0].script = txgen.push(_sig(tx, canon, value, 0, k, rng))
    out.append(("p2pk_canonical", [tx], [(0, 0, canon, value)]))
    ks = _keys(rng, 2)
    script = txgen.multisig_script(1, [k.pub for k in ks])
    tx = txgen._ms_tx(rng)
    value = rng.randrange(1, 2**40)
    tx.inputs[0].script = b"\x00" + txgen.push(_sig(tx, script, value, 0, ks[0], rng))
    out.append(("one_of_two_one_sig", [tx], [(0, 0, script, value)]))
    return out


def _oracle(coracle, txs, jobs):
    from test_sighash_oracle import multisig_verdicts
    return multisig_verdicts(coracle, txs, jobs, None)


@pytest.mark.parametrize("name", sorted(CHOSEN))
def test_reading_oracle(coracle, name):
    case = {nm: (t, j) for nm, t, j in reading_cases()}[name]
    assert _oracle(coracle, *case) == [CHOSEN[name]], (name, "alternative reading gives", ALT[name])


def test_reading_controls_verify(coracle):
    for name, txs, jobs in _controls():
        assert _oracle(coracle, txs, jobs) == [True], name


@pytest.mark.gpu
def test_reading_gpu_both_entry_points(coracle):
    """Every reading case (and the controls) through the host entry point
    and the device one, in one batch: the kernels take the chosen reading."""
    import numpy as np
    import torch
    import hkv
    from test_gpu_sighash import _device_verify_std
    cases = reading_cases() + _controls()
    raw, jobs, want, names = [], [], [], []
    for name, txs, js in cases:
        base = len(raw)
        raw += [sh.tx_serialize(t) for t in txs]
        jobs += [(t + base, i, p, v) for (t, i, p, v) in js]
        want += [CHOSEN.get(name, True)] * len(js)
        names += [name] * len(js)
    with hkv.Verifier(hkv.VerifierConfig(device_ids=[0], flags=1)) as ver:
        got = hkv.verify_std_inputs(ver, raw, jobs, None)
        assert got == want, [(n, g, w) for n, g, w in zip(names, got, want) if g != w]
        assert _device_verify_std(torch, ver, raw, jobs, None) == want
    assert np.array(want).sum() == 3  # the empty-item case and the two controls
