"""CPU tests: pin the sighash / standard-input oracle (oracle/sighash_oracle.py)
before trusting it.

* the reference's own fixtures: the 15 coinbase txs of
  /root/reference/test/Haskoin/NodeSpec.hs:282-340 (tests/golden/ref_blocks.bin)
  decode and re-serialise byte-exactly, and SHA-256d of each equals its
  block's merkle root (1-tx blocks);
* the published BIP143 "native P2WPKH" example (tests/golden/bip143_p2wpkh.json):
  BIP143 intermediate hashes + sighash; HASH160; and the example's published
  signatures verify against OUR legacy sighash (P2PK input 0) and OUR BIP143
  sighash (P2WPKH input 1), end to end through std_input;
* RIPEMD-160 published vectors;
* DER decode edge rules of secp256k1_ecdsa_signature_parse_der;
* legacy sighash corner semantics (SINGLE bug, ANYONECANPAY, codeseparators).
"""
import json
import os
import random

import pytest

import secp256k1_oracle as o
import sighash_oracle as sh
import txgen
from conftest import GOLDEN, oracle_batch


@pytest.fixture(scope="module")
def bip143():
    return json.load(open(os.path.join(GOLDEN, "bip143_p2wpkh.json")))


def signed_bip143_tx(b):
    tx = sh.tx_parse(bytes.fromhex(b["unsigned_tx"]))
    i0, i1 = b["inputs"]
    tx.inputs[0].script = txgen.push(bytes.fromhex(i0["sig"]))
    tx.witness = [[], [bytes.fromhex(i1["sig"]), bytes.fromhex(i1["pubkey"])]]
    return tx


def test_ripemd160_vectors(bip143):
    for msg, hx in bip143["ripemd160_vectors"].items():
        assert sh.ripemd160(msg.encode()).hex() == hx


def test_bip143_example_hashes(bip143):
    tx = sh.tx_parse(bytes.fromhex(bip143["unsigned_tx"]))
    assert sh.tx_serialize(tx).hex() == bip143["unsigned_tx"]
    exp = bip143["input1_sighash_all"]
    hp, hs, ho = sh.bip143_parts(tx, 1, sh.SIGHASH_ALL)
    assert (hp.hex(), hs.hex(), ho.hex()) == (exp["hashPrevouts"], exp["hashSequence"], exp["hashOutputs"])
    i1 = bip143["inputs"][1]
    h20 = bytes.fromhex(i1["script_pubkey"])[2:]
    assert sh.hash160(bytes.fromhex(i1["pubkey"])) == h20
    m = sh.sighash_forkid(tx, sh.p2pkh_script(h20), i1["value"], 1, sh.SIGHASH_ALL)
    assert m.hex() == exp["sigHash"]


def test_bip143_example_signatures_pin_both_sighash_forms(bip143):
    """Published signatures verify only against the exact sighash bytes."""
    tx = signed_bip143_tx(bip143)
    raw = sh.tx_serialize(tx)
    assert sh.tx_serialize(sh.tx_parse(raw)) == raw  # witness form round trip
    for i, inp in enumerate(bip143["inputs"]):
        spk = bytes.fromhex(inp["script_pubkey"])
        si = sh.std_input(tx, i, spk, inp["value"])
        assert si.ok, inp["kind"]
        assert o.verify_hash_sig(si.msg32, si.r, si.s, o.pubkey_parse(si.pubkey))
        # any other value / index / sighash type breaks it
        bad = sh.std_input(tx, i, spk, inp["value"] + 1)
        if inp["kind"] == "p2wpkh":
            assert not o.verify_hash_sig(bad.msg32, bad.r, bad.s, o.pubkey_parse(bad.pubkey))
        m2 = sh.sighash_legacy(tx, spk, inp["value"], i, 0x81)
        assert not o.verify_hash_sig(m2, si.r, si.s, o.pubkey_parse(si.pubkey))


def test_reference_coinbase_txs_roundtrip_to_merkle_root():
    """NodeSpec.hs:282-340 fixture blocks: tx codec + SHA-256d txid."""
    raw = open(os.path.join(GOLDEN, "ref_blocks.bin"), "rb").read()
    off, n = 0, 0
    while off < len(raw):
        hdr = raw[off:off + 80]
        assert raw[off + 80] == 1
        st = off + 81
        # the coinbase is the rest of the block up to the next header: find it by decoding
        tx = None
        for end in range(st + 10, len(raw) + 1):
            try:
                tx = sh.tx_parse(raw[st:end])
                break
            except (ValueError, KeyError):
                continue
        assert tx is not None
        ser = sh.tx_serialize(tx)
        assert raw[st:st + len(ser)] == ser
        assert sh.sha256d(ser) == hdr[36:68]
        assert len(tx.inputs) == 1 and tx.inputs[0].prev_hash == b"\0" * 32
        off = st + len(ser)
        n += 1
    assert n == 15


def test_der_rules():
    r, s = 0x1234, 0x5678
    good = sh.der_encode(r, s)
    assert sh.sig_parse_der(good) == (r, s)
    assert sh.sig_parse_der(good + b"\x00") is None                       # trailing garbage
    assert sh.sig_parse_der(b"\x30\x81" + bytes([len(good) - 2]) + good[2:]) is None  # long-form len < 128
    assert sh.sig_parse_der(b"\x30\x80" + good[2:]) is None               # indefinite
    assert sh.sig_parse_der(b"\x30\x06\x02\x02\x00\x01\x02\x01\x01") is None  # excessive 0x00 padding
    assert sh.sig_parse_der(b"\x30\x06\x02\x02\xff\x80\x02\x01\x01") is None  # excessive 0xff padding
    assert sh.sig_parse_der(b"\x30\x06\x02\x01\x80\x02\x01\x01") == (0, 1)   # negative -> overflow -> 0
    assert sh.sig_parse_der(b"\x30\x05\x02\x00\x02\x01\x01") is None      # zero-length integer
    n_enc = sh.der_encode(o.N, 1)
    assert sh.sig_parse_der(n_enc) == (0, 1)                              # r >= n -> 0
    big = b"\x02\x21\x00" + b"\xff" * 32
    assert sh.sig_parse_der(b"\x30" + bytes([len(big) + 3]) + big + b"\x02\x01\x01") == (0, 1)
    assert sh.decode_strict_sig(n_enc) is None                            # zero r rejected
    assert sh.decode_strict_sig(sh.der_encode(1, o.N - 1)) is None        # high S rejected
    assert sh.decode_strict_sig(sh.der_encode(1, o.N // 2)) == (1, o.N // 2)
    assert sh.decode_tx_sig(good + b"\x01") == (r, s, 1)
    assert sh.decode_tx_sig(good + b"\x04") is None                       # unknown hashtype
    assert sh.decode_tx_sig(good + b"\x41") is None                       # forkid on a no-forkid net
    assert sh.decode_tx_sig(good + b"\x41", forkid=0) == (r, s, 0x41)


def test_legacy_corner_cases():
    rng = random.Random(3)
    tx = txgen.rand_tx(rng, 3, 2)
    code = sh.p2pkh_script(b"\x11" * 20)
    assert sh.sighash_legacy(tx, code, 0, 2, 3) == sh.ONE                 # SINGLE, i >= #outs
    assert sh.sighash_legacy(tx, code, 0, 2, 0x83) == sh.ONE
    assert sh.sighash_legacy(tx, code, 0, 1, 3) != sh.ONE
    # unknown base types behave as ALL apart from the appended type word
    a = sh.tx_serialize(sh.Tx(tx.version, [sh.TxIn(t.prev_hash, t.prev_index, code if j == 0 else b"", t.sequence)
                                          for j, t in enumerate(tx.inputs)], tx.outputs, [], tx.locktime), False)
    assert sh.sighash_legacy(tx, code, 0, 0, 4) == sh.sha256d(a + (4).to_bytes(4, "little"))
    # codeseparators are removed, but not inside push data
    assert sh.strip_codeseparators(b"\xab\x01\xab\xab") == b"\x01\xab"
    assert sh.strip_codeseparators(b"\xab\x4c\xff") == b"\xab\x4c\xff"    # unparseable: verbatim
    # ANYONECANPAY commits to only input i: other inputs' data does not matter
    tx2 = txgen.rand_tx(rng, 3, 2)
    tx2.inputs[1] = tx.inputs[1]
    tx2.outputs, tx2.version, tx2.locktime = tx.outputs, tx.version, tx.locktime
    assert sh.sighash_legacy(tx, code, 0, 1, 0x81) == sh.sighash_legacy(tx2, code, 0, 1, 0x81)
    assert sh.sighash_legacy(tx, code, 0, 1, 0x01) != sh.sighash_legacy(tx2, code, 0, 1, 0x01)
    # forkid dispatch only on a fork-id network
    assert sh.sighash_legacy(tx, code, 7, 1, 0x41, forkid=0) == sh.sighash_forkid(tx, code, 7, 1, 0x41, 0)
    assert sh.sighash_legacy(tx, code, 7, 1, 0x41) != sh.sighash_forkid(tx, code, 7, 1, 0x41)


def test_std_block_generator_is_valid():
    rng = random.Random(11)
    keys = [txgen.Key(rng.randrange(1, o.N), compressed=(k % 4 != 0)) for k in range(8)]
    txs, jobs = txgen.std_block(rng, 10, keys, p2wpkh_share=0.4, p2pk_share=0.2, p2sh_share=0.2)
    assert any(len(p) == 23 for _, _, p, _ in jobs)  # P2SH-P2WPKH present
    for t, i, prev, val in jobs:
        tx = sh.tx_parse(sh.tx_serialize(txs[t]))
        si = sh.std_input(tx, i, prev, val)
        assert si.ok
        assert o.verify_hash_sig(si.msg32, si.r, si.s, o.pubkey_parse(si.pubkey))
        assert len(sh.std_input_record(tx, i, prev, val)) == 168


def test_p2sh_p2wpkh_rules():
    """P2SH-P2WPKH (BIP16 + BIP141): one push of the 00 14 <h20> redeem script
    hashing to the P2SH hash, witness [sig, pubkey], BIP143 sighash over the
    P2PKH scriptCode of the program; every deviation rejects."""
    rng = random.Random(12)
    keys = [txgen.Key(rng.randrange(1, o.N)) for _ in range(4)]
    txs, jobs = txgen.std_block(rng, 12, keys, p2wpkh_share=0.0, p2pk_share=0.0, p2sh_share=1.0)
    t, i, prev, val = jobs[0]
    tx = sh.tx_parse(sh.tx_serialize(txs[t]))
    good = sh.std_input(tx, i, prev, val)
    assert good.ok and o.verify_hash_sig(good.msg32, good.r, good.s, o.pubkey_parse(good.pubkey))
    rd = sh._push_items(tx.inputs[i].script)[0]
    # the same spend seen as native P2WPKH of the program signs the same message
    tx2 = sh.tx_parse(sh.tx_serialize(tx))
    tx2.inputs[i].script = b""
    assert sh.std_input(tx2, i, sh.p2wpkh_script(rd[2:]), val).msg32 == good.msg32
    for script in (b"", tx.inputs[i].script * 2, txgen.push(rd + b"\x00"), txgen.push(b"\x00\x14" + bytes(20)),
                   b"\x51" + tx.inputs[i].script):
        bad = sh.tx_parse(sh.tx_serialize(tx))
        bad.inputs[i].script = script
        assert not sh.std_input(bad, i, prev, val).ok
    # a non-minimal push of the redeem script is still one data push
    nm = sh.tx_parse(sh.tx_serialize(tx))
    nm.inputs[i].script = b"\x4c\x16" + rd
    assert sh.std_input(nm, i, prev, val).ok
    assert not sh.std_input(tx, i, prev[:-1] + b"\x88", val).ok



MS_VALID = {"valid", "empty_skip_ok", "mixed_sighash"}


def multisig_verdicts(coracle, txs, jobs, forkid):
    """Oracle verdicts of multisig (or any standard) inputs: candidate records
    checked by the C restatement in HASKOIN mode, keys by pubkey_parse."""
    out = []
    for (t, i, prev, val) in jobs:
        out.append(sh.verify_std_input(txs[t], i, prev, val, forkid,
                                       lambda recs: oracle_batch(coracle, b"".join(recs), 1),
                                       lambda k: o.pubkey_parse(k) is not None))
    return out


@pytest.mark.parametrize("forkid", [None, 0])
def test_multisig_oracle_labels(coracle, forkid):
    """The restated countMulSig walk (haskoin-core verifyStdInput, PayMulSig
    branch) on bare and P2SH m-of-n inputs: signatures in key order verify;
    swapped, missing, extra (count m + 1 != m), wrong-key, high-S, unknown
    hashtype, undecodable items (also past the n-th), a missing / non-OP_0
    dummy, m > n, a wrong key count, an off-curve or hybrid key, a PUSHDATA1
    key push (non-canonical, the template limit) and a wrong redeem hash all
    fail; an empty item consumes exactly one key."""
    rng = random.Random(77 + (forkid or 0))
    keys = [txgen.Key(rng.randrange(1, o.N), compressed=(k % 4 != 0)) for k in range(24)]
    txs, jobs, names = txgen.multisig_cases(rng, keys, forkid)
    got = multisig_verdicts(coracle, txs, jobs, forkid)
    want = [nm.split("-", 2)[2] in MS_VALID for nm in names]
    bad = [(names[k], got[k]) for k in range(len(jobs)) if got[k] != want[k]]
    assert not bad, bad[:10]
    assert sum(want) > 80 and len(want) - sum(want) > 400
    assert {nm.split("-")[0] for nm in names} == {"bare", "p2sh", "p2wsh", "p2sh_p2wsh"}


def test_multisig_candidate_order_and_walk():
    """Candidates are (j, k) for nonempty j < min(#sigs, n), k = j..n-1, in
    that order; the walk consumes a key per step and a signature per match
    or empty item."""
    ms = sh.MultiSig(2, [b"a", b"b", b"c"], [None, (1, 1, 1), (1, 1, 1), (1, 1, 1)], [sh.ZERO32] * 3)
    assert ms.candidates() == [(1, 1), (1, 2), (2, 2)]
    # empty sig 0 consumes key a; sig 1 matches b; sig 2 vs c
    assert ms.resolve([True, False, True], [True] * 3)
    assert not ms.resolve([True, False, False], [True] * 3)
    assert not ms.resolve([False, True, True], [True] * 3)      # sig 1 matches c: sig 2 has no key left
    assert not ms.resolve([True, False, True], [True, False, True])
    ms1 = sh.MultiSig(1, [b"a", b"b"], [(1, 1, 1)], [sh.ZERO32])
    assert ms1.candidates() == [(0, 0), (0, 1)]
    assert ms1.resolve([False, True], [True, True])


@pytest.mark.parametrize("forkid", [None, 0])
def test_wrapped_single_sig_oracle_labels(coracle, forkid):
    """P2SH-P2PK / P2SH-P2PKH (legacy sighash over the redeem script) and
    P2WSH-P2PK / P2WSH-P2PKH, native and P2SH-nested (BIP143 over the
    witness script): valid spends verify; a corrupted signature, a wrong
    script hash, an extra or missing stack item, a wrong key and high S fail;
    NONE and ANYONECANPAY|SINGLE signatures made over their own sighash
    verify."""
    rng = random.Random(99 + (forkid or 0))
    keys = [txgen.Key(rng.randrange(1, o.N), compressed=(k % 3 != 0)) for k in range(8)]
    txs, jobs, names = txgen.wrapped_single_cases(rng, keys, forkid)
    got = multisig_verdicts(coracle, txs, jobs, forkid)
    # (a P2PK stack has no key: "wrong_pub" changes nothing there)
    want = [nm.split("-")[1] in ("valid", "other_sighash", "acp_single")
            or (nm.split("-")[1] == "wrong_pub" and nm.split("-")[0].endswith("_p2pk")) for nm in names]
    bad = [(names[k], got[k]) for k in range(len(jobs)) if got[k] != want[k]]
    assert not bad, bad[:10]
