"""CPU oracle (TEST INFRASTRUCTURE ONLY) — pure-Python restatement of the
reference stack's signature-hash and standard-input functions.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker. The product path
(``haskoin-node_amd/``) never imports it.

What it restates. None of these
functions is in ``/root/reference``; they live in haskoin-core-1.1.0, pinned at
``/root/reference/stack.yaml:10`` / ``stack.yaml.lock:14-20`` [dep]:

* ``tx_parse`` / ``tx_serialize`` — the ``Tx`` wire codec (BIP144 segwit
  marker/flag, witness stacks), ``Haskoin.Transaction.Common``; the reference
  decodes peer messages with it at ``src/Haskoin/Node/Peer.hs:270``.
* ``sighash_legacy``  — ``Haskoin.Script.SigHash.txSigHash``: copy of the tx
  with every scriptSig empty except input i = scriptCode with OP_CODESEPARATOR
  ops removed; NONE drops all outputs; SINGLE keeps i blank outputs
  (value 2^64-1, empty script) plus output i; NONE/SINGLE zero the other
  inputs' sequence; ANYONECANPAY keeps only input i; unknown base types
  behave as ALL; SINGLE with i >= #outputs signs the integer one
  (``01 00 .. 00``). The copy is re-serialised (canonical varints, no
  witnesses), then ``LE32(sighash)`` and SHA-256d. On a network with a fork id
  and the FORKID flag (0x40) it dispatches to the BIP143 form.
* ``sighash_forkid``  — ``txSigHashForkId``: the BIP143 preimage
  (hashPrevouts / hashSequence / hashOutputs with the ANYONECANPAY / NONE /
  SINGLE zeroing rules) and ``sigHashAddNetworkId`` (sh | forkid << 8).
* ``sha256d``         — ``Haskoin.Crypto.Hash.doubleSHA256`` (a9); pinned by
  the header hashes the reference's tests assert
  (``test/Haskoin/NodeSpec.hs:180-218``, tests/test_oracle.py).
* ``ripemd160`` / ``hash160`` — ``Haskoin.Crypto.Hash.addressHash``
  (RIPEMD160 . SHA256); restated here because this image's OpenSSL 3 does not
  expose RIPEMD-160 through hashlib.
* ``decode_strict_sig`` / ``std_input`` — ``Haskoin.Crypto.Signature``
  ``decodeStrictSig`` (libsecp256k1 ``secp256k1_ecdsa_signature_parse_der``
  + r, s != 0 + low S), ``Haskoin.Script.SigHash.decodeTxSig`` and
  ``Haskoin.Transaction.Builder.verifyStdInput`` restricted to the P2PK,
  P2PKH and P2WPKH templates (HASH160(pubkey) must equal the template's hash;
  a P2WPKH input's scriptSig must be empty and its witness exactly
  [sig, pubkey]).

Parity status: SHA-256d is pinned by the reference's fixture
hashes, and the wire codec by re-serialising the fixture coinbase txs to their
merkle roots. Both sighash forms, HASH160 and the DER decode are pinned by the
published BIP143 "native P2WPKH" example (tests/golden/bip143_p2wpkh.json):
hashPrevouts / hashSequence / hashOutputs and the BIP143 sighash of input 1
reproduce, HASH160 of its key equals its witness program, and the example's
published signatures verify against our legacy sighash of its P2PK input 0 and
our BIP143 sighash of input 1. RIPEMD-160 is also pinned by its published test
vectors. Beyond those vectors the rules follow the published definitions above
(the reference's own fixture blocks are coinbase-only).
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

SIGHASH_ALL = 1
SIGHASH_NONE = 2
SIGHASH_SINGLE = 3
SIGHASH_FORKID = 0x40
SIGHASH_ANYONECANPAY = 0x80

ONE = b"\x01" + b"\x00" * 31
ZERO32 = b"\x00" * 32
OP_CODESEPARATOR = 0xAB


def sha256d(data: bytes) -> bytes:
    return hashlib.sha256(hashlib.sha256(data).digest()).digest()


# --- RIPEMD-160 --------------------------------------------------------------
_RL = [list(range(16)),
       [7, 4, 13, 1, 10, 6, 15, 3, 12, 0, 9, 5, 2, 14, 11, 8],
       [3, 10, 14, 4, 9, 15, 8, 1, 2, 7, 0, 6, 13, 11, 5, 12],
       [1, 9, 11, 10, 0, 8, 12, 4, 13, 3, 7, 15, 14, 5, 6, 2],
       [4, 0, 5, 9, 7, 12, 2, 10, 14, 1, 3, 8, 11, 6, 15, 13]]
_RR = [[5, 14, 7, 0, 9, 2, 11, 4, 13, 6, 15, 8, 1, 10, 3, 12],
       [6, 11, 3, 7, 0, 13, 5, 10, 14, 15, 8, 12, 4, 9, 1, 2],
       [15, 5, 1, 3, 7, 14, 6, 9, 11, 8, 12, 2, 10, 0, 4, 13],
       [8, 6, 4, 1, 3, 11, 15, 0, 5, 12, 2, 13, 9, 7, 10, 14],
       [12, 15, 10, 4, 1, 5, 8, 7, 6, 2, 13, 14, 0, 3, 9, 11]]
_SL = [[11, 14, 15, 12, 5, 8, 7, 9, 11, 13, 14, 15, 6, 7, 9, 8],
       [7, 6, 8, 13, 11, 9, 7, 15, 7, 12, 15, 9, 11, 7, 13, 12],
       [11, 13, 6, 7, 14, 9, 13, 15, 14, 8, 13, 6, 5, 12, 7, 5],
       [11, 12, 14, 15, 14, 15, 9, 8, 9, 14, 5, 6, 8, 6, 5, 12],
       [9, 15, 5, 11, 6, 8, 13, 12, 5, 12, 13, 14, 11, 8, 5, 6]]
_SR = [[8, 9, 9, 11, 13, 15, 15, 5, 7, 7, 8, 11, 14, 14, 12, 6],
       [9, 13, 15, 7, 12, 8, 9, 11, 7, 7, 12, 7, 6, 15, 13, 11],
       [9, 7, 15, 11, 8, 6, 6, 14, 12, 13, 5, 14, 13, 13, 7, 5],
       [15, 5, 8, 11, 14, 14, 6, 14, 6, 9, 12, 9, 12, 5, 15, 8],
       [8, 5, 12, 9, 12, 5, 14, 6, 8, 13, 6, 5, 15, 13, 11, 11]]
_KL = [0x00000000, 0x5A827999, 0x6ED9EBA1, 0x8F1BBCDC, 0xA953FD4E]
_KR = [0x50A28BE6, 0x5C4DD124, 0x6D703EF3, 0x7A6D76E9, 0x00000000]
_M32 = 0xFFFFFFFF


def _rol(x: int, n: int) -> int:
    return ((x << n) | (x >> (32 - n))) & _M32


def _rf(j: int, x: int, y: int, z: int) -> int:
    if j == 0:
        return x ^ y ^ z
    if j == 1:
        return (x & y) | (~x & z & _M32)
    if j == 2:
        return (x | (~y & _M32)) ^ z
    if j == 3:
        return (x & z) | (y & ~z & _M32)
    return x ^ (y | (~z & _M32))


def ripemd160(data: bytes) -> bytes:
    h = [0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0]
    msg = data + b"\x80" + b"\x00" * ((55 - len(data)) % 64) + (8 * len(data)).to_bytes(8, "little")
    for blk in range(0, len(msg), 64):
        x = [int.from_bytes(msg[blk + 4 * k:blk + 4 * k + 4], "little") for k in range(16)]
        al, bl, cl, dl, el = h
        ar, br, cr, dr, er = h
        for rnd in range(5):
            for k in range(16):
                t = (_rol((al + _rf(rnd, bl, cl, dl) + x[_RL[rnd][k]] + _KL[rnd]) & _M32, _SL[rnd][k]) + el) & _M32
                al, el, dl, cl, bl = el, dl, _rol(cl, 10), bl, t
                t = (_rol((ar + _rf(4 - rnd, br, cr, dr) + x[_RR[rnd][k]] + _KR[rnd]) & _M32, _SR[rnd][k]) + er) & _M32
                ar, er, dr, cr, br = er, dr, _rol(cr, 10), br, t
        t = (h[1] + cl + dr) & _M32
        h[1] = (h[2] + dl + er) & _M32
        h[2] = (h[3] + el + ar) & _M32
        h[3] = (h[4] + al + br) & _M32
        h[4] = (h[0] + bl + cr) & _M32
        h[0] = t
    return b"".join(v.to_bytes(4, "little") for v in h)


def hash160(data: bytes) -> bytes:
    return ripemd160(hashlib.sha256(data).digest())


# --- wire codec --------------------------------------------------------------

def put_varint(n: int) -> bytes:
    if n < 0xFD:
        return bytes([n])
    if n <= 0xFFFF:
        return b"\xfd" + n.to_bytes(2, "little")
    if n <= 0xFFFFFFFF:
        return b"\xfe" + n.to_bytes(4, "little")
    return b"\xff" + n.to_bytes(8, "little")


def get_varint(b: bytes, off: int) -> Tuple[int, int]:
    """VarInt decoding (non-canonical encodings are accepted)."""
    if off >= len(b):
        raise ValueError("truncated varint")
    t = b[off]
    if t < 0xFD:
        return t, off + 1
    w = {0xFD: 2, 0xFE: 4, 0xFF: 8}[t]
    if off + 1 + w > len(b):
        raise ValueError("truncated varint")
    return int.from_bytes(b[off + 1:off + 1 + w], "little"), off + 1 + w


@dataclass
class TxIn:
    prev_hash: bytes   # 32 bytes, wire order
    prev_index: int
    script: bytes
    sequence: int

    def outpoint(self) -> bytes:
        return self.prev_hash + self.prev_index.to_bytes(4, "little")


@dataclass
class TxOut:
    value: int
    script: bytes

    def serialize(self) -> bytes:
        return self.value.to_bytes(8, "little") + put_varint(len(self.script)) + self.script


@dataclass
class Tx:
    version: int
    inputs: List[TxIn]
    outputs: List[TxOut]
    witness: List[List[bytes]] = field(default_factory=list)
    locktime: int = 0


def tx_serialize(tx: Tx, with_witness: bool = True) -> bytes:
    seg = with_witness and any(len(w) for w in tx.witness)
    out = [tx.version.to_bytes(4, "little")]
    if seg:
        out.append(b"\x00\x01")
    out.append(put_varint(len(tx.inputs)))
    for ti in tx.inputs:
        out += [ti.outpoint(), put_varint(len(ti.script)), ti.script, ti.sequence.to_bytes(4, "little")]
    out.append(put_varint(len(tx.outputs)))
    out += [to.serialize() for to in tx.outputs]
    if seg:
        for k in range(len(tx.inputs)):
            stack = tx.witness[k] if k < len(tx.witness) else []
            out.append(put_varint(len(stack)))
            for item in stack:
                out += [put_varint(len(item)), item]
    out.append(tx.locktime.to_bytes(4, "little"))
    return b"".join(out)


def tx_parse(b: bytes) -> Tx:
    """Wire decoding (BIP144 marker 00 01 selects the witness form)."""
    if len(b) < 10:
        raise ValueError("short tx")
    ver = int.from_bytes(b[0:4], "little")
    off = 4
    seg = b[4] == 0 and b[5] == 1
    if seg:
        off = 6
    nin, off = get_varint(b, off)
    ins = []
    for _ in range(nin):
        if off + 36 > len(b):
            raise ValueError("truncated input")
        ph, pi = b[off:off + 32], int.from_bytes(b[off + 32:off + 36], "little")
        sl, off = get_varint(b, off + 36)
        if off + sl + 4 > len(b):
            raise ValueError("truncated input")
        sc = b[off:off + sl]
        off += sl
        seq = int.from_bytes(b[off:off + 4], "little")
        off += 4
        ins.append(TxIn(ph, pi, sc, seq))
    nout, off = get_varint(b, off)
    outs = []
    for _ in range(nout):
        if off + 8 > len(b):
            raise ValueError("truncated output")
        v = int.from_bytes(b[off:off + 8], "little")
        sl, off = get_varint(b, off + 8)
        if off + sl > len(b):
            raise ValueError("truncated output")
        outs.append(TxOut(v, b[off:off + sl]))
        off += sl
    wit: List[List[bytes]] = []
    if seg:
        for _ in range(nin):
            k, off = get_varint(b, off)
            items = []
            for _ in range(k):
                il, off = get_varint(b, off)
                if off + il > len(b):
                    raise ValueError("truncated witness")
                items.append(b[off:off + il])
                off += il
            wit.append(items)
    if off + 4 != len(b):
        raise ValueError("bad length")
    lock = int.from_bytes(b[off:off + 4], "little")
    return Tx(ver, ins, outs, wit, lock)


# --- scripts -----------------------------------------------------------------

def script_ops(script: bytes) -> Optional[List[Tuple[int, int]]]:
    """Split a script into (start, end) byte ranges per op; None if a push runs
    past the end (haskoin's Script cannot hold such a script)."""
    ops, off = [], 0
    while off < len(script):
        op = script[off]
        st = off
        off += 1
        if 1 <= op <= 75:
            off += op
        elif op == 0x4C:
            if off + 1 > len(script):
                return None
            off += 1 + script[off]
        elif op == 0x4D:
            if off + 2 > len(script):
                return None
            off += 2 + int.from_bytes(script[off:off + 2], "little")
        elif op == 0x4E:
            if off + 4 > len(script):
                return None
            off += 4 + int.from_bytes(script[off:off + 4], "little")
        if off > len(script):
            return None
        ops.append((st, off))
    return ops


def strip_codeseparators(script: bytes) -> bytes:
    """filter (/= OP_CODESEPARATOR) . scriptOps (txSigHash)."""
    ops = script_ops(script)
    if ops is None:
        return script
    return b"".join(script[a:b] for a, b in ops if not (b - a == 1 and script[a] == OP_CODESEPARATOR))


# --- txSigHash / txSigHashForkId (a7, a8) --------------------------------------

def _base(sh: int) -> int:
    return sh & 0x1F


def sighash_legacy(tx: Tx, script_code: bytes, value: int, i: int, sh: int,
                   forkid: Optional[int] = None) -> bytes:
    """haskoin-core txSigHash. ``forkid`` None = network without a fork id."""
    if forkid is not None and (sh & SIGHASH_FORKID):
        return sighash_forkid(tx, script_code, value, i, sh, forkid)
    out = strip_codeseparators(script_code)
    base = _base(sh)
    is_all = base not in (SIGHASH_NONE, SIGHASH_SINGLE)  # ALL or unknown
    if sh & SIGHASH_ANYONECANPAY:
        ti = tx.inputs[i]
        ins = [TxIn(ti.prev_hash, ti.prev_index, out, ti.sequence)]
    else:
        ins = []
        for j, ti in enumerate(tx.inputs):
            sc = out if j == i else b""
            seq = ti.sequence if (is_all or j == i) else 0
            ins.append(TxIn(ti.prev_hash, ti.prev_index, sc, seq))
    if is_all:
        outs = list(tx.outputs)
    elif base == SIGHASH_NONE:
        outs = []
    else:
        if i >= len(tx.outputs):
            return ONE
        outs = [TxOut(0xFFFFFFFFFFFFFFFF, b"") for _ in range(i)] + [tx.outputs[i]]
    pre = tx_serialize(Tx(tx.version, ins, outs, [], tx.locktime), with_witness=False)
    return sha256d(pre + (sh & 0xFFFFFFFF).to_bytes(4, "little"))


def bip143_parts(tx: Tx, i: int, sh: int) -> Tuple[bytes, bytes, bytes]:
    """(hashPrevouts, hashSequence, hashOutputs) of txSigHashForkId."""
    acp = bool(sh & SIGHASH_ANYONECANPAY)
    base = _base(sh)
    single, none = base == SIGHASH_SINGLE, base == SIGHASH_NONE
    hp = ZERO32 if acp else sha256d(b"".join(ti.outpoint() for ti in tx.inputs))
    hs = ZERO32 if (acp or single or none) else sha256d(
        b"".join(ti.sequence.to_bytes(4, "little") for ti in tx.inputs))
    if not single and not none:
        ho = sha256d(b"".join(to.serialize() for to in tx.outputs))
    elif single and i < len(tx.outputs):
        ho = sha256d(tx.outputs[i].serialize())
    else:
        ho = ZERO32
    return hp, hs, ho


def sighash_forkid(tx: Tx, script_code: bytes, value: int, i: int, sh: int, forkid: Optional[int] = None) -> bytes:
    """haskoin-core txSigHashForkId (BIP143 preimage)."""
    hp, hs, ho = bip143_parts(tx, i, sh)
    ti = tx.inputs[i]
    shn = sh if forkid is None else (sh | (forkid << 8))
    pre = (tx.version.to_bytes(4, "little") + hp + hs + ti.outpoint() + put_varint(len(script_code)) + script_code
           + value.to_bytes(8, "little") + ti.sequence.to_bytes(4, "little") + ho + tx.locktime.to_bytes(4, "little")
           + (shn & 0xFFFFFFFF).to_bytes(4, "little"))
    return sha256d(pre)


KIND_LEGACY = 0   # txSigHash
KIND_FORKID = 1   # txSigHashForkId


def sighash_job(tx: Tx, kind: int, script_code: bytes, value: int, i: int, sh: int,
                forkid: Optional[int] = None) -> bytes:
    if kind == KIND_FORKID:
        return sighash_forkid(tx, script_code, value, i, sh, forkid)
    return sighash_legacy(tx, script_code, value, i, sh, forkid)


# --- DER signatures (secp256k1_ecdsa_signature_parse_der + decodeStrictSig) ---

N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


def _der_len(b: bytes, off: int, end: int) -> Tuple[Optional[int], int]:
    """libsecp256k1 secp256k1_der_read_len: definite, minimal length."""
    if off >= end:
        return None, off
    b1 = b[off]
    off += 1
    if b1 == 0xFF:
        return None, off
    if (b1 & 0x80) == 0:
        return b1, off
    lenleft = b1 & 0x7F
    if lenleft == 0:
        return None, off          # indefinite length
    if lenleft > end - off:
        return None, off
    if b[off] == 0:
        return None, off          # not the shortest encoding
    if lenleft > 8:
        return None, off
    ret = 0
    for _ in range(lenleft):
        ret = (ret << 8) | b[off]
        off += 1
    if ret > end - off:
        return None, off
    if ret < 128:
        return None, off          # should have used the short form
    return ret, off


def _der_int(b: bytes, off: int, end: int) -> Tuple[Optional[int], int]:
    """secp256k1_der_parse_integer: overflow -> value 0 (parse still ok)."""
    if off >= end or b[off] != 0x02:
        return None, off
    off += 1
    rlen, off = _der_len(b, off, end)
    if rlen is None or rlen == 0 or rlen > end - off:
        return None, off
    if b[off] == 0x00 and rlen > 1 and (b[off + 1] & 0x80) == 0:
        return None, off          # excessive 0x00 padding
    if b[off] == 0xFF and rlen > 1 and (b[off + 1] & 0x80) == 0x80:
        return None, off          # excessive 0xFF padding
    overflow = bool(b[off] & 0x80)  # negative
    if b[off] == 0:
        off += 1
        rlen -= 1
    if rlen > 32:
        overflow = True
    v = 0 if overflow else int.from_bytes(b[off:off + rlen], "big")
    if v >= N:
        v = 0
    return v, off + rlen


def sig_parse_der(b: bytes) -> Optional[Tuple[int, int]]:
    """secp256k1_ecdsa_signature_parse_der (overflowing integers parse as 0)."""
    end = len(b)
    if end == 0 or b[0] != 0x30:
        return None
    rlen, off = _der_len(b, 1, end)
    if rlen is None or rlen != end - off:
        return None
    r, off = _der_int(b, off, end)
    if r is None:
        return None
    s, off = _der_int(b, off, end)
    if s is None:
        return None
    if off != end:
        return None
    return r, s


def der_encode(r: int, s: int) -> bytes:
    def enc(v: int) -> bytes:
        b = v.to_bytes(32, "big").lstrip(b"\x00") or b"\x00"
        if b[0] & 0x80:
            b = b"\x00" + b
        return b"\x02" + bytes([len(b)]) + b
    body = enc(r) + enc(s)
    return b"\x30" + bytes([len(body)]) + body


def decode_strict_sig(b: bytes) -> Optional[Tuple[int, int]]:
    """haskoin-core decodeStrictSig: DER parse, r != 0, s != 0, low S."""
    rs = sig_parse_der(b)
    if rs is None:
        return None
    r, s = rs
    if r == 0 or s == 0 or s > N // 2:
        return None
    return rs


def is_sighash_unknown(sh: int) -> bool:
    return _base(sh) not in (SIGHASH_ALL, SIGHASH_NONE, SIGHASH_SINGLE)


def decode_tx_sig(b: bytes, forkid: Optional[int] = None) -> Optional[Tuple[int, int, int]]:
    """haskoin-core decodeTxSig: strict sig + trailing sighash byte."""
    if len(b) < 1:
        return None
    rs = decode_strict_sig(b[:-1])
    if rs is None:
        return None
    sh = b[-1]
    if is_sighash_unknown(sh):
        return None
    if forkid is None and (sh & SIGHASH_FORKID):
        return None
    return rs[0], rs[1], sh


def p2pkh_script(h20: bytes) -> bytes:
    return b"\x76\xa9\x14" + h20 + b"\x88\xac"


def p2wpkh_script(h20: bytes) -> bytes:
    return b"\x00\x14" + h20


def _push_items(script: bytes) -> Optional[List[bytes]]:
    """The data of a script made only of data pushes (opcodes 1..78); None for
    anything else (OP_0 and OP_1..16 are not data pushes here)."""
    ops = script_ops(script)
    if ops is None:
        return None
    items = []
    for a, e in ops:
        op = script[a]
        if 1 <= op <= 75:
            items.append(script[a + 1:e])
        elif op == 0x4C:
            items.append(script[a + 2:e])
        elif op == 0x4D:
            items.append(script[a + 3:e])
        elif op == 0x4E:
            items.append(script[a + 5:e])
        else:
            return None
    return items


def pubkey_bytes_ok(pub: bytes) -> bool:
    """haskoin PubKeyI deserialisation: 02/03 + 32 bytes or 04 + 64 bytes
    (hybrid 06/07 is not a haskoin public key); curve checks happen in the
    ECDSA record parse."""
    return (len(pub) == 33 and pub[0] in (2, 3)) or (len(pub) == 65 and pub[0] == 4)


@dataclass
class StdInput:
    """What the batch path needs from one standard input."""
    ok: bool                 # template / encoding checks passed
    msg32: bytes = ZERO32
    r: int = 0
    s: int = 0
    pubkey: bytes = b""


def std_input(tx: Tx, i: int, prev_script: bytes, value: int, forkid: Optional[int] = None) -> StdInput:
    """The non-ECDSA half of verifyStdInput for the single-signature
    templates: P2PK, P2PKH, P2WPKH, P2SH-wrapped P2PK / P2PKH / P2WPKH,
    P2WSH-wrapped P2PK / P2PKH (native and P2SH-nested): template match,
    strict signature decode, HASH160 / SHA-256 script checks and sighash. The input verifies iff ok and verifyHashSig(msg32, (r, s), pubkey).
    P2PK is matched in its direct-push forms (21 <33> ac, 41 <65> ac)."""
    if i >= len(tx.inputs):
        return StdInput(False)
    if (len(prev_script) == 35 and prev_script[0] == 0x21 or len(prev_script) == 67 and prev_script[0] == 0x41) \
            and prev_script[-1] == 0xAC:
        pub = prev_script[1:-1]
        items = _push_items(tx.inputs[i].script)
        if items is None or len(items) != 1 or not pubkey_bytes_ok(pub):
            return StdInput(False)
        ts = decode_tx_sig(items[0], forkid)
        if ts is None:
            return StdInput(False)
        r, s, sh = ts
        m = sighash_legacy(tx, prev_script, value, i, sh, forkid)
        return StdInput(True, m, r, s, pub)
    if len(prev_script) == 25 and prev_script[:3] == b"\x76\xa9\x14" and prev_script[23:] == b"\x88\xac":
        items = _push_items(tx.inputs[i].script)
        if items is None or len(items) != 2:
            return StdInput(False)
        sig, pub = items
        ts = decode_tx_sig(sig, forkid)
        if ts is None or not pubkey_bytes_ok(pub) or hash160(pub) != prev_script[3:23]:
            return StdInput(False)
        r, s, sh = ts
        m = sighash_legacy(tx, prev_script, value, i, sh, forkid)
        return StdInput(True, m, r, s, pub)
    if len(prev_script) == 22 and prev_script[:2] == b"\x00\x14":
        wit = tx.witness[i] if i < len(tx.witness) else []
        if len(tx.inputs[i].script) != 0 or len(wit) != 2:
            return StdInput(False)
        sig, pub = wit
        ts = decode_tx_sig(sig, forkid)
        if ts is None or not pubkey_bytes_ok(pub) or hash160(pub) != prev_script[2:22]:
            return StdInput(False)
        r, s, sh = ts
        m = sighash_forkid(tx, p2pkh_script(prev_script[2:22]), value, i, sh, forkid)
        return StdInput(True, m, r, s, pub)
    if len(prev_script) == 34 and prev_script[:2] == b"\x00\x20":
        # P2WSH (haskoin verifySegwitInput, PayWitnessScriptHash): empty
        # scriptSig, witness = stack ++ [witness script], SHA-256(witness
        # script) == the program, the script a PayPK / PayPKHash (multisig:
        # std_multisig), BIP143 sighash over the witness script.
        if len(tx.inputs[i].script) != 0:
            return StdInput(False)
        wit = tx.witness[i] if i < len(tx.witness) else []
        return _p2wsh_single(tx, i, prev_script[2:34], wit, value, forkid)
    if len(prev_script) == 23 and prev_script[:2] == b"\xa9\x14" and prev_script[22] == 0x87:
        # P2SH (BIP16): the scriptSig's last push is the redeem script, whose
        # HASH160 is the script hash. Nested segwit (haskoin's
        # nestedScriptOutput branch): the scriptSig is exactly that push of
        # 00 14 <h20> (P2SH-P2WPKH: then as P2WPKH of the program) or
        # 00 20 <h32> (P2SH-P2WSH). Otherwise verifyLegacyInput on the redeem
        # script: PayPK with [sig], PayPKHash with [sig, pub] before it, legacy
        # sighash over the redeem script (multisig: std_multisig). No reference
        # data holds a P2SH spend: parity unpinned.
        items = _push_items(tx.inputs[i].script)
        if items is None or not items or hash160(items[-1]) != prev_script[2:22]:
            return StdInput(False)
        rd, stack = items[-1], items[:-1]
        wit = tx.witness[i] if i < len(tx.witness) else []
        if len(rd) == 22 and rd[:2] == b"\x00\x14":
            if stack or len(wit) != 2:
                return StdInput(False)
            sig, pub = wit
            ts = decode_tx_sig(sig, forkid)
            if ts is None or not pubkey_bytes_ok(pub) or hash160(pub) != rd[2:22]:
                return StdInput(False)
            r, s, sh = ts
            m = sighash_forkid(tx, p2pkh_script(rd[2:22]), value, i, sh, forkid)
            return StdInput(True, m, r, s, pub)
        if len(rd) == 34 and rd[:2] == b"\x00\x20":
            if stack:
                return StdInput(False)
            return _p2wsh_single(tx, i, rd[2:34], wit, value, forkid)
        return _script_single(tx, i, rd, stack, value, forkid, False)
    return StdInput(False)


def _p2pk_key(script: bytes) -> Optional[bytes]:
    """The key of a direct-push P2PK script (21 <33> ac / 41 <65> ac)."""
    if (len(script) == 35 and script[0] == 0x21 or len(script) == 67 and script[0] == 0x41) and script[-1] == 0xAC:
        return script[1:-1]
    return None


def _script_single(tx: Tx, i: int, code: bytes, stack: List[bytes], value: int, forkid: Optional[int],
                   segwit: bool) -> StdInput:
    """A P2PK / P2PKH script (redeem or witness script) with its stack:
    [sig] / [sig, pub]; sighash over `code`, legacy or BIP143."""
    pub = _p2pk_key(code)
    if pub is not None:
        if len(stack) != 1 or not pubkey_bytes_ok(pub):
            return StdInput(False)
        sig = stack[0]
    elif len(code) == 25 and code[:3] == b"\x76\xa9\x14" and code[23:] == b"\x88\xac":
        if len(stack) != 2:
            return StdInput(False)
        sig, pub = stack
        if not pubkey_bytes_ok(pub) or hash160(pub) != code[3:23]:
            return StdInput(False)
    else:
        return StdInput(False)
    ts = decode_tx_sig(sig, forkid)
    if ts is None:
        return StdInput(False)
    r, s, sh = ts
    m = sighash_forkid(tx, code, value, i, sh, forkid) if segwit else sighash_legacy(tx, code, value, i, sh, forkid)
    return StdInput(True, m, r, s, pub)


def _p2wsh_single(tx: Tx, i: int, prog: bytes, wit: List[bytes], value: int, forkid: Optional[int]) -> StdInput:
    if not wit or hashlib.sha256(wit[-1]).digest() != prog:
        return StdInput(False)
    return _script_single(tx, i, wit[-1], list(wit[:-1]), value, forkid, True)


def _record(msg32: bytes, r: int, s: int, pub: bytes) -> bytes:
    rec = msg32 + r.to_bytes(32, "big") + s.to_bytes(32, "big") + bytes([len(pub)]) + pub.ljust(65, b"\x00")
    return rec.ljust(168, b"\x00")


def std_input_record(tx: Tx, i: int, prev_script: bytes, value: int, forkid: Optional[int] = None) -> bytes:
    """The 168-byte verify record the device extractor must produce (an
    all-zero record when the template checks fail, and for multisig inputs,
    which are resolved from candidate records instead: std_multisig)."""
    si = std_input(tx, i, prev_script, value, forkid)
    if not si.ok:
        return b"\x00" * 168
    return _record(si.msg32, si.r, si.s, si.pubkey)


# --- multisig: bare and P2SH (haskoin-core verifyStdInput's PayMulSig branch) ----
#
# haskoin-core-1.1.0 [dep, stack.yaml:10] Haskoin.Transaction.Builder:
#   verifyStdInput ... (PayMulSig pubs r) (SpendMulSig sigs) = countMulSig ... pubs sigs == r
#   countMulSig' _ [] _ = 0
#   countMulSig' _ _ [] = 0
#   countMulSig' h (_ : pubs) (TxSignatureEmpty : sigs) = countMulSig' h pubs sigs
#   countMulSig' h (PubKeyI pub _ : pubs) sigs@(TxSignature sig sh : sigs')
#     | verifyHashSig (h sh) sig pub = 1 + countMulSig' h pubs sigs'
#     | otherwise = countMulSig' h pubs sigs
# with h sh = txSigHash net tx (encodeOutput so) value i sh. Decoding
# (Haskoin.Script.Standard): the output must be OP_m <keys> OP_n
# OP_CHECKMULTISIG, 1 <= m <= n <= 16, n keys that deserialise as PubKeyI
# (02/03 + 32 bytes or 04 + 64 bytes AND a point on the curve, importPubKey);
# the input must be OP_0 followed by items that are OP_0 / empty pushes
# (TxSignatureEmpty) or decodeTxSig-valid signatures (any other item fails the
# whole decode). P2SH: the scriptSig's last op is a push of the redeem script,
# which must decode as the multisig output and whose HASH160 is the P2SH hash;
# the scriptCode is then the redeem script. Parity with the reference stack is
# unpinned by data (the reference fixtures hold no multisig); deliberate limit
# shared with P2PK: keys must be direct pushes (21 / 41), so encodeOutput's
# canonical re-encoding equals the script bytes.

def multisig_template(script: bytes) -> Optional[Tuple[int, List[bytes]]]:
    """(m, keys) of a canonical OP_m <k_1..k_n> OP_n OP_CHECKMULTISIG script."""
    L = len(script)
    if L < 3 or script[-1] != 0xAE:
        return None
    m, n = script[0] - 0x50, script[-2] - 0x50
    if not (1 <= m <= 16 and 1 <= n <= 16 and m <= n):
        return None
    keys, off = [], 1
    while off < L - 2:
        op = script[off]
        if op not in (0x21, 0x41) or off + 1 + op > L - 2:
            return None
        k = script[off + 1:off + 1 + op]
        if not pubkey_bytes_ok(k):
            return None
        keys.append(k)
        off += 1 + op
    if off != L - 2 or len(keys) != n:
        return None
    return m, keys


def _multisig_items(script: bytes, p2sh: bool) -> Optional[Tuple[List[Optional[bytes]], bytes]]:
    """scriptSig -> (items, redeem): items are None for OP_0 / empty pushes;
    the first op must be OP_0 (the CHECKMULTISIG dummy, haskoin matchMulSig)."""
    ops = script_ops(script)
    if ops is None or len(ops) < (2 if p2sh else 1) or script[ops[0][0]] != 0x00:
        return None
    redeem = b""
    body = ops[1:]
    if p2sh:
        last = _push_items(script[ops[-1][0]:ops[-1][1]])
        if last is None or len(last) != 1:
            return None
        redeem = last[0]
        body = ops[1:-1]
    items: List[Optional[bytes]] = []
    for a, e in body:
        if script[a] == 0x00:
            items.append(None)
            continue
        d = _push_items(script[a:e])
        if d is None:
            return None
        items.append(d[0] if d[0] else None)
    return items, redeem


@dataclass
class MultiSig:
    """A structurally valid multisig input: what the batch path verifies."""
    m: int
    keys: List[bytes]
    sigs: List[Optional[Tuple[int, int, int]]]   # (r, s, sighash) or None (empty)
    msgs: List[bytes]                             # sighash of sig j (j < min(#sigs, n)), ZERO32 if empty

    def candidates(self) -> List[Tuple[int, int]]:
        """(sig j, key k) pairs the CHECKMULTISIG walk can compare, in the
        device's order: nonempty j < min(#sigs, n), then k = j .. n-1."""
        n = len(self.keys)
        return [(j, k) for j in range(min(len(self.sigs), n)) if self.sigs[j] is not None for k in range(j, n)]

    def candidate_records(self) -> List[bytes]:
        return [_record(self.msgs[j], self.sigs[j][0], self.sigs[j][1], self.keys[k]) for j, k in self.candidates()]

    def key_records(self) -> List[bytes]:
        return [_record(ZERO32, 0, 0, k) for k in self.keys]

    def resolve(self, cand_ok: List[bool], keys_ok: List[bool]) -> bool:
        """countMulSig' over the candidate verdicts; all keys must be points."""
        if not all(keys_ok):
            return False
        idx = {c: v for c, v in zip(self.candidates(), cand_ok)}
        count, j = 0, 0
        for k in range(len(self.keys)):
            if j >= len(self.sigs):
                break
            if self.sigs[j] is None:
                j += 1
                continue
            if idx[(j, k)]:
                count += 1
                j += 1
        return count == self.m


def std_multisig(tx: Tx, i: int, prev_script: bytes, value: int, forkid: Optional[int] = None
                 ) -> Optional[MultiSig]:
    """Decode a bare, P2SH, P2WSH or P2SH-P2WSH multisig input (None: not
    one, or it fails to decode, i.e. verifyStdInput is False). Segwit forms:
    witness = [empty dummy] ++ items ++ [witness script], SHA-256(witness
    script) == the program, empty scriptSig (nested: exactly the push of
    00 20 <h32>), BIP143 sighash over the witness script; items follow the
    scriptSig rules (empty = TxSignatureEmpty)."""
    if i >= len(tx.inputs):
        return None
    ss = tx.inputs[i].script
    wit = tx.witness[i] if i < len(tx.witness) else []
    p2sh = len(prev_script) == 23 and prev_script[:2] == b"\xa9\x14" and prev_script[22] == 0x87
    prog = None
    if len(prev_script) == 34 and prev_script[:2] == b"\x00\x20":
        if ss:
            return None
        prog = prev_script[2:34]
    elif p2sh:
        pushes = _push_items(ss)
        if pushes is not None and len(pushes) == 1 and len(pushes[0]) == 34 and pushes[0][:2] == b"\x00\x20":
            if hash160(pushes[0]) != prev_script[2:22]:
                return None
            prog = pushes[0][2:34]
    segwit = prog is not None
    if segwit:
        if len(wit) < 2 or wit[0] != b"" or hashlib.sha256(wit[-1]).digest() != prog:
            return None
        code = wit[-1]
        items: List[Optional[bytes]] = [x if x else None for x in wit[1:-1]]
    elif p2sh:
        it = _multisig_items(ss, True)
        if it is None:
            return None
        items, code = it
        if hash160(code) != prev_script[2:22]:
            return None
    else:
        code = prev_script
        it = _multisig_items(ss, False)
        if it is None:
            return None
        items = it[0]
    tmpl = multisig_template(code)
    if tmpl is None:
        return None
    m, keys = tmpl
    sigs: List[Optional[Tuple[int, int, int]]] = []
    for item in items:
        if item is None:
            sigs.append(None)
            continue
        ts = decode_tx_sig(item, forkid)
        if ts is None:
            return None
        sigs.append(ts)
    msgs = []
    for j in range(min(len(sigs), len(keys))):
        if sigs[j] is None:
            msgs.append(ZERO32)
        elif segwit:
            msgs.append(sighash_forkid(tx, code, value, i, sigs[j][2], forkid))
        else:
            msgs.append(sighash_legacy(tx, code, value, i, sigs[j][2], forkid))
    return MultiSig(m, keys, sigs, msgs)


def verify_std_input(tx: Tx, i: int, prev_script: bytes, value: int, forkid: Optional[int], verify_records,
                     key_ok) -> bool:
    """Full verifyStdInput verdict. verify_records(list of records) -> list of
    bools (HASKOIN-mode ECDSA, e.g. the C oracle); key_ok(pubkey bytes) ->
    importPubKey succeeds."""
    ms = std_multisig(tx, i, prev_script, value, forkid)
    if ms is not None:
        cands = ms.candidate_records()
        return ms.resolve(list(verify_records(cands)) if cands else [], [key_ok(k) for k in ms.keys])
    rec = std_input_record(tx, i, prev_script, value, forkid)
    return bool(verify_records([rec])[0])
