"""Seeded transaction / block generators for the sighash and standard-input
tests (test infrastructure: builds inputs with the oracle's codec and signs
with the oracle's curve arithmetic)."""
from __future__ import annotations

import random
from typing import List, Optional, Tuple

import secp256k1_oracle as o
import sighash_oracle as sh


def rand_script(rng: random.Random, n: int) -> bytes:
    return bytes(rng.randrange(256) for _ in range(n))


def rand_tx(rng: random.Random, nin: int, nout: int, segwit: bool = False, big_scripts: bool = False) -> sh.Tx:
    ins = []
    for _ in range(nin):
        slen = rng.choice([0, 1, 25, 106, 107, 139]) if not big_scripts else rng.choice([0, 252, 253, 300, 70000])
        ins.append(sh.TxIn(rand_script(rng, 32), rng.randrange(2**32), rand_script(rng, slen),
                           rng.choice([0xFFFFFFFF, 0xFFFFFFFE, rng.randrange(2**32)])))
    outs = []
    for _ in range(nout):
        slen = rng.choice([0, 22, 23, 25, 34, 80]) if not big_scripts else rng.choice([0, 252, 253, 1000])
        outs.append(sh.TxOut(rng.randrange(2**64), rand_script(rng, slen)))
    wit = []
    if segwit:
        for _ in range(nin):
            wit.append([rand_script(rng, rng.choice([0, 33, 72])) for _ in range(rng.randrange(3))])
        if not any(len(w) for w in wit):
            wit[0] = [b"\x01"]
    return sh.Tx(rng.choice([1, 2, 0xFFFFFFFF]), ins, outs, wit, rng.randrange(2**32))


def rand_sighash(rng: random.Random) -> int:
    return rng.choice([1, 1, 1, 2, 3, 0x81, 0x82, 0x83, 0x41, 0xC1, 0x43, 0, 4, 0x1F, 0x21, 0xFF,
                       0x12345601, rng.randrange(2**32)])


def rand_code(rng: random.Random) -> bytes:
    kind = rng.randrange(6)
    if kind == 0:
        return sh.p2pkh_script(rand_script(rng, 20))
    if kind == 1:   # with OP_CODESEPARATORs between ops
        return b"\xab" + sh.p2pkh_script(rand_script(rng, 20))[:3] + rand_script(rng, 20) + b"\xab\x88\xac\xab"
    if kind == 2:   # 0xab inside push data must survive
        return b"\x05\xab\xab\xab\xab\xab\xab\x4c\x02\xab\x01\xab"
    if kind == 3:   # truncated push: not a parseable script, kept verbatim
        return b"\xab\x4c\xff\xab"
    if kind == 4:
        return b""
    return rand_script(rng, rng.choice([1, 10, 300]))


# --- signing (private keys; RFC6979 is not needed for tests) -----------------

def sign(msg32: bytes, d: int, k: int) -> Tuple[int, int]:
    R = o.point_mul(k, o.G)
    r = R[0] % o.N
    s = pow(k, -1, o.N) * (int.from_bytes(msg32, "big") + r * d) % o.N
    if s > o.N // 2:
        s = o.N - s
    return r, s


class Key:
    def __init__(self, d: int, compressed: bool = True):
        self.d = d
        self.q = o.point_mul(d, o.G)
        self.pub = o.pubkey_serialize(self.q, compressed)
        self.h160 = sh.hash160(self.pub)


def push(data: bytes) -> bytes:
    n = len(data)
    if n <= 75:
        return bytes([n]) + data
    if n <= 255:
        return b"\x4c" + bytes([n]) + data
    return b"\x4d" + n.to_bytes(2, "little") + data


def std_block(rng: random.Random, n_tx: int, keys: List[Key], forkid: Optional[int] = None,
              p2wpkh_share: float = 0.6, p2pk_share: float = 0.0, p2sh_share: float = 0.0,
              nin_choices=(1, 1, 2, 2, 3)):
    """A synthetic block mix: every tx spends 1-3 (nin_choices) standard
    prevouts (P2WPKH / P2PKH / P2PK / P2SH-P2WPKH) and pays 2 outputs,
    SIGHASH_ALL (| FORKID on a fork-id network). Returns (txs, jobs) with
    jobs = [(tx index, input, prevout script, value)]."""
    txs, jobs = [], []
    shbyte = 0x41 if forkid is not None else 0x01
    for t in range(n_tx):
        nin = rng.choice(list(nin_choices))
        kinds, ks, vals = [], [], []
        ins = []
        for _ in range(nin):
            u = rng.random()
            kind = "p2wpkh" if u < p2wpkh_share else ("p2pk" if u < p2wpkh_share + p2pk_share else (
                "p2sh" if u < p2wpkh_share + p2pk_share + p2sh_share else "p2pkh"))
            kinds.append(kind)
            ks.append(rng.choice(keys))
            vals.append(rng.randrange(1, 2**50))
            ins.append(sh.TxIn(rand_script(rng, 32), rng.randrange(4), b"", 0xFFFFFFFF))
        outs = [sh.TxOut(rng.randrange(1, 2**40), sh.p2pkh_script(rand_script(rng, 20))) for _ in range(2)]
        tx = sh.Tx(rng.choice([1, 2]), ins, outs, [[] for _ in range(nin)], rng.randrange(600000))
        prevs = []
        for j in range(nin):
            k = ks[j]
            if kinds[j] == "p2wpkh":
                prevs.append(sh.p2wpkh_script(k.h160))
            elif kinds[j] == "p2pk":
                prevs.append(push(k.pub) + b"\xac")
            elif kinds[j] == "p2sh":
                prevs.append(b"\xa9\x14" + sh.hash160(sh.p2wpkh_script(k.h160)) + b"\x87")
            else:
                prevs.append(sh.p2pkh_script(k.h160))
        for j in range(nin):
            k = ks[j]
            if kinds[j] in ("p2wpkh", "p2sh"):
                m = sh.sighash_forkid(tx, sh.p2pkh_script(k.h160), vals[j], j, shbyte, forkid)
            else:
                m = sh.sighash_legacy(tx, prevs[j], vals[j], j, shbyte, forkid)
            r, s = sign(m, k.d, rng.randrange(1, o.N))
            sig = sh.der_encode(r, s) + bytes([shbyte])
            if kinds[j] == "p2wpkh":
                tx.witness[j] = [sig, k.pub]
            elif kinds[j] == "p2sh":
                tx.witness[j] = [sig, k.pub]
                tx.inputs[j].script = push(sh.p2wpkh_script(k.h160))
            elif kinds[j] == "p2pk":
                tx.inputs[j].script = push(sig)
            else:
                tx.inputs[j].script = push(sig) + push(k.pub)
        txs.append(tx)
        for j in range(nin):
            jobs.append((t, j, prevs[j], vals[j]))
    return txs, jobs


# --- multisig (bare and P2SH) -------------------------------------------------

def multisig_script(m: int, pubs: List[bytes]) -> bytes:
    return bytes([0x50 + m]) + b"".join(push(p) for p in pubs) + bytes([0x50 + len(pubs), 0xAE])


def p2sh_script(redeem: bytes) -> bytes:
    return b"\xa9\x14" + sh.hash160(redeem) + b"\x87"


def _ms_tx(rng: random.Random) -> sh.Tx:
    ins = [sh.TxIn(rand_script(rng, 32), rng.randrange(4), b"", 0xFFFFFFFF) for _ in range(rng.choice([1, 2]))]
    outs = [sh.TxOut(rng.randrange(1, 2**40), sh.p2pkh_script(rand_script(rng, 20))) for _ in range(2)]
    return sh.Tx(1, ins, outs, [[] for _ in ins], rng.randrange(600000))


OFF_CURVE = b"\x02" + (5).to_bytes(32, "big")   # x = 5: x^3 + 7 is not a square mod p


def multisig_cases(rng: random.Random, keys: List[Key], forkid: Optional[int] = None,
                   wraps=("bare", "p2sh", "p2wsh", "p2sh_p2wsh")):
    """Bare, P2SH, P2WSH and P2SH-P2WSH m-of-n inputs, valid and adversarial
    (one input per tx, signatures made against the real scriptCode: legacy
    for bare / P2SH, BIP143 over the witness script for the segwit forms).
    Returns (txs, jobs, names) with jobs = (tx index, input, prevout script,
    value); the verdict of each is decided by the oracle
    (sighash_oracle.verify_std_input), not here."""
    import hashlib
    txs, jobs, names = [], [], []
    base_sh = 0x41 if forkid is not None else 0x01
    shapes = [(1, 1), (1, 2), (2, 2), (2, 3), (3, 5), (1, 3), (4, 7), (15, 15), (1, 16)]
    variants = ["valid", "swap", "fewer", "extra", "wrong_key", "empty_skip_ok", "empty_skip_bad", "no_dummy",
                "dummy_op1", "m_gt_n", "n_mismatch", "off_curve_other", "hybrid_key", "pushdata1_key",
                "bad_redeem_hash", "mixed_sighash", "bad_der_after_n", "trailing_op", "high_s", "all_empty",
                "unknown_hashtype", "sig_past_end"]
    for (m, n) in shapes:
        for wrap in wraps:
            seg = wrap in ("p2wsh", "p2sh_p2wsh")
            for var in variants:
                if var in ("swap",) and m < 2:
                    continue
                if var in ("extra", "empty_skip_ok", "empty_skip_bad") and m == n:
                    continue
                if wrap == "bare" and var == "bad_redeem_hash":
                    continue
                if seg and var in ("trailing_op", "sig_past_end"):
                    continue
                ks = rng.sample(keys, n)
                pubs = [k.pub for k in ks]
                mm = m
                if var == "off_curve_other":
                    pubs = pubs[:]
                    pubs[-1] = OFF_CURVE
                elif var == "hybrid_key":
                    q = ks[-1].q
                    pubs = pubs[:-1] + [bytes([6 | (q[1] & 1)]) + q[0].to_bytes(32, "big") + q[1].to_bytes(32, "big")]
                script = multisig_script(mm, pubs)
                if var == "m_gt_n":
                    script = bytes([0x50 + n + 1]) + script[1:] if n < 16 else b"\x61" + script[1:]
                elif var == "n_mismatch":
                    script = script[:-2] + bytes([0x50 + (n - 1 if n > 1 else 2), 0xAE])
                elif var == "pushdata1_key":
                    script = bytes([0x50 + m]) + b"\x4c" + bytes([len(pubs[0])]) + pubs[0] + \
                        b"".join(push(p) for p in pubs[1:]) + bytes([0x50 + n, 0xAE])
                wprog = b"\x00\x20" + hashlib.sha256(script).digest()
                if wrap == "bare":
                    prev = script
                elif wrap == "p2sh":
                    prev = p2sh_script(script)
                elif wrap == "p2wsh":
                    prev = wprog
                else:
                    prev = p2sh_script(wprog)
                if var == "bad_redeem_hash":
                    prev = b"\xa9\x14" + bytes(20) + b"\x87" if wrap != "p2wsh" else b"\x00\x20" + bytes(32)
                tx = _ms_tx(rng)
                i = rng.randrange(len(tx.inputs))
                value = rng.randrange(1, 2**50)
                idx = sorted(rng.sample(range(n), m))
                if var == "extra":
                    idx = sorted(rng.sample(range(n), m + 1))
                elif var == "fewer":
                    idx = idx[:-1]
                elif var == "empty_skip_ok":   # an empty item consumes key 0; the signers come later
                    idx = sorted(rng.sample(range(1, n), m))
                elif var == "empty_skip_bad":  # ... but key 0 itself signs: the empty item skips it
                    idx = [0] + sorted(rng.sample(range(1, n), m - 1)) if m > 1 else [0]
                shs = [base_sh] * len(idx)
                if var == "mixed_sighash":
                    shs = [rng.choice([1, 2, 3, 0x81, 0x82, 0x83]) | (0x40 if forkid is not None else 0)
                           for _ in idx]
                if var == "unknown_hashtype" and shs:
                    shs[0] = 0x04
                items = []
                for k, shb in zip(idx, shs):
                    if seg:
                        msg = sh.sighash_forkid(tx, script, value, i, shb, forkid)
                    else:
                        msg = sh.sighash_legacy(tx, script, value, i, shb, forkid)
                    d = ks[k].d
                    if var == "wrong_key" and k == idx[-1]:
                        d = rng.randrange(1, o.N)
                    r, s = sign(msg, d, rng.randrange(1, o.N))
                    if var == "high_s" and k == idx[0]:
                        s = o.N - s
                    items.append(sh.der_encode(r, s) + bytes([shb]))
                if var == "swap":
                    items[0], items[1] = items[1], items[0]
                if var in ("empty_skip_ok", "empty_skip_bad"):
                    items = [b""] + items
                if var == "all_empty":
                    items = [b""] * m
                if var == "bad_der_after_n":
                    items = items + [b""] * (n - len(items)) + [b"\x30\x02\x01\x01\x01"]
                if seg:
                    dummy = [b"\x01"] if var == "dummy_op1" else ([] if var == "no_dummy" else [b""])
                    tx.witness[i] = dummy + items + [script]
                    tx.inputs[i].script = push(wprog) if wrap == "p2sh_p2wsh" else b""
                else:
                    sig_part = b"".join(b"\x00" if not x else push(x) for x in items)
                    if var == "sig_past_end":
                        sig_part = sig_part + b"\x4c\x50\x30"
                    dummy = b"\x51" if var == "dummy_op1" else (b"" if var == "no_dummy" else b"\x00")
                    ss = dummy + sig_part
                    if var == "trailing_op":
                        ss += b"\x75"   # OP_DROP: not a push, the decode fails
                    if wrap == "p2sh":
                        ss += push(script)
                    tx.inputs[i].script = ss
                txs.append(tx)
                jobs.append((len(txs) - 1, i, prev, value))
                names.append(f"{wrap}-{m}of{n}-{var}")
    return txs, jobs, names


def wrapped_single_cases(rng: random.Random, keys: List[Key], forkid: Optional[int] = None):
    """Single-signature inputs behind P2SH / P2WSH (haskoin verifyStdInput's
    ScriptHashInput and PayWitnessScriptHash branches): P2SH-P2PK,
    P2SH-P2PKH, P2WSH-P2PK, P2WSH-P2PKH, P2SH-P2WSH-P2PK, P2SH-P2WSH-P2PKH,
    valid and mutated. Returns (txs, jobs, names); verdicts by the oracle."""
    import hashlib
    txs, jobs, names = [], [], []
    base_sh = 0x41 if forkid is not None else 0x01
    kinds = ["p2sh_p2pk", "p2sh_p2pkh", "p2wsh_p2pk", "p2wsh_p2pkh", "p2sh_p2wsh_p2pk", "p2sh_p2wsh_p2pkh"]
    variants = ["valid", "valid", "bad_sig", "bad_hash", "extra_item", "missing_item", "wrong_pub", "high_s",
                "other_sighash", "acp_single"]
    for kind in kinds:
        for var in variants:
            k = rng.choice(keys)
            inner = push(k.pub) + b"\xac" if kind.endswith("_p2pk") else sh.p2pkh_script(k.h160)
            seg = "p2wsh" in kind
            wprog = b"\x00\x20" + hashlib.sha256(inner).digest()
            if kind.startswith("p2sh_p2wsh"):
                prev = p2sh_script(wprog)
            elif kind.startswith("p2wsh"):
                prev = wprog
            else:
                prev = p2sh_script(inner)
            if var == "bad_hash":
                prev = prev[:5] + bytes([prev[5] ^ 1]) + prev[6:]
            tx = _ms_tx(rng)
            i = rng.randrange(len(tx.inputs))
            value = rng.randrange(1, 2**50)
            shb = base_sh
            if var == "other_sighash":
                shb = 0x02 | (0x40 if forkid is not None else 0)
            if var == "acp_single":
                shb = 0x83 | (0x40 if forkid is not None else 0)
            msg = sh.sighash_forkid(tx, inner, value, i, shb, forkid) if seg else \
                sh.sighash_legacy(tx, inner, value, i, shb, forkid)
            r, s = sign(msg, k.d, rng.randrange(1, o.N))
            if var == "high_s":
                s = o.N - s
            sig = sh.der_encode(r, s) + bytes([shb])
            if var == "bad_sig":
                sig = sig[:6] + bytes([sig[6] ^ 4]) + sig[7:]
            pub = k.pub if var != "wrong_pub" else Key(rng.randrange(1, o.N)).pub
            stack = [sig] if kind.endswith("_p2pk") else [sig, pub]
            if var == "extra_item":
                stack = stack + [b"\x01"]
            if var == "missing_item":
                stack = stack[:-1]
            if seg:
                tx.witness[i] = stack + [inner]
                tx.inputs[i].script = push(wprog) if kind.startswith("p2sh") else b""
            else:
                tx.inputs[i].script = b"".join(push(x) for x in stack) + push(inner)
            txs.append(tx)
            jobs.append((len(txs) - 1, i, prev, value))
            names.append(f"{kind}-{var}")
    return txs, jobs, names
