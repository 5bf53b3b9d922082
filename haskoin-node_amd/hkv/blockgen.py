"""Synthetic blocks for the benchmark and the tests.

* ``make_block`` — the mainnet-shaped block mix (BASELINE.json configs[2],
  SURVEY.md §8(d) config 3): 2,000 txs (default), each spending 1-3 prevouts
  (60% P2WPKH / 40% P2PKH) and paying 2 P2PKH outputs, SIGHASH_ALL, no fork id.
* ``make_p2pkh_block`` — the CPU-reference block (BASELINE.json configs[0],
  SURVEY.md §8(d) config 1): 2,000 txs x 2 P2PKH inputs x 2 P2PKH outputs =
  4,000 signatures, compressed keys from a pool of 4,096, SIGHASH_ALL, low S,
  seed 0x484B5631.
 Keys, sighashes and
signatures come from libhkv's device hooks (hkv_gen_keys_device,
hkv_sighash, hkv_gen_sign_device): the sighash of a tx does not depend on its
scriptSigs / witnesses, so the block is hashed as a skeleton, signed, then
assembled. Data is synthetic (no network, no chain): outpoints and output
hashes are random bytes.
"""
from __future__ import annotations

import ctypes
import random
import struct
from typing import List, Tuple

import numpy as np

from .lib import HKV_SIGHASH_FORKID, HKV_SIGHASH_LEGACY
from .sighash import tx_sig_hash_batch

SEED = 0x484B5633
P2PKH_SEED = 0x484B5631


def varint(n: int) -> bytes:
    if n < 0xFD:
        return bytes([n])
    if n <= 0xFFFF:
        return b"\xfd" + struct.pack("<H", n)
    return b"\xfe" + struct.pack("<I", n)


def push(data: bytes) -> bytes:
    return bytes([len(data)]) + data if len(data) <= 75 else b"\x4c" + bytes([len(data)]) + data


def der(r: bytes, s: bytes) -> bytes:
    def enc(v: bytes) -> bytes:
        v = v.lstrip(b"\0") or b"\0"
        if v[0] & 0x80:
            v = b"\0" + v
        return b"\x02" + bytes([len(v)]) + v
    body = enc(r) + enc(s)
    return b"\x30" + bytes([len(body)]) + body


def p2pkh(h20: bytes) -> bytes:
    return b"\x76\xa9\x14" + h20 + b"\x88\xac"


def serialize(version, ins, outs, wit, lock) -> bytes:
    seg = any(wit)
    b = [struct.pack("<I", version)]
    if seg:
        b.append(b"\x00\x01")
    b.append(varint(len(ins)))
    for (op, script, seq) in ins:
        b += [op, varint(len(script)), script, struct.pack("<I", seq)]
    b.append(varint(len(outs)))
    for (val, script) in outs:
        b += [struct.pack("<Q", val), varint(len(script)), script]
    if seg:
        for items in wit:
            b.append(varint(len(items)))
            for it in items:
                b += [varint(len(it)), it]
    b.append(struct.pack("<I", lock))
    return b"".join(b)


def make_block(verifier, torch, n_tx: int = 2000, seed: int = SEED, n_keys: int = 4096,
               p2wpkh_share: float = 0.6, inputs_per_tx=(1, 1, 2, 2, 3)
               ) -> Tuple[List[bytes], List[Tuple[int, int, bytes, int]]]:
    """Returns (serialised txs, inputs) with inputs = (tx, input index, prevout
    scriptPubKey, prevout value): the arguments of verify_std_inputs."""
    rng = random.Random(seed)
    priv = torch.zeros(n_keys * 32, dtype=torch.uint8, device="cuda")
    pub = torch.zeros(n_keys * 33, dtype=torch.uint8, device="cuda")
    h160 = torch.zeros(n_keys * 20, dtype=torch.uint8, device="cuda")
    verifier.gen_keys_device(0, seed, n_keys, priv.data_ptr(), pub.data_ptr(), h160.data_ptr())
    torch.cuda.synchronize()
    pubs, hs = pub.cpu().numpy().tobytes(), h160.cpu().numpy().tobytes()

    txs, meta, jobs, key_idx = [], [], [], []
    for t in range(n_tx):
        nin = rng.choice(inputs_per_tx)
        ins, kinds = [], []
        for j in range(nin):
            k = rng.randrange(n_keys)
            seg = rng.random() < p2wpkh_share
            value = rng.randrange(1000, 2**45)
            ins.append((rng.randbytes(32) + struct.pack("<I", rng.randrange(4)), b"", 0xFFFFFFFF))
            kinds.append((seg, k, value))
            h = hs[20 * k:20 * k + 20]
            jobs.append((t, j, p2pkh(h), value, 1, HKV_SIGHASH_FORKID if seg else HKV_SIGHASH_LEGACY))
            key_idx.append(k)
        outs = [(rng.randrange(546, 2**40), p2pkh(rng.randbytes(20))) for _ in range(2)]
        version, lock = rng.choice([1, 2]), rng.randrange(800000)
        txs.append(serialize(version, ins, outs, [], lock))
        meta.append((version, ins, outs, lock, kinds))
    msgs, status = tx_sig_hash_batch(verifier, txs, jobs)
    assert not any(status), "skeleton txs must parse"
    d_msg = torch.from_numpy(np.frombuffer(b"".join(msgs), dtype=np.uint8).copy()).cuda()
    d_idx = torch.tensor(key_idx, dtype=torch.int32, device="cuda")
    d_sig = torch.zeros(len(jobs) * 64, dtype=torch.uint8, device="cuda")
    verifier.gen_sign_device(0, seed ^ 0x5167, len(jobs), priv.data_ptr(), d_idx.data_ptr(), d_msg.data_ptr(), 32,
                             d_sig.data_ptr())
    torch.cuda.synchronize()
    sigs = d_sig.cpu().numpy().tobytes()

    out_txs, inputs, q = [], [], 0
    for t, (version, ins, outs, lock, kinds) in enumerate(meta):
        new_ins, wit = [], []
        for j, (seg, k, value) in enumerate(kinds):
            sig = der(sigs[64 * q:64 * q + 32], sigs[64 * q + 32:64 * q + 64]) + b"\x01"
            pk, h = pubs[33 * k:33 * k + 33], hs[20 * k:20 * k + 20]
            if seg:
                new_ins.append((ins[j][0], b"", ins[j][2]))
                wit.append([sig, pk])
                inputs.append((t, j, b"\x00\x14" + h, value))
            else:
                new_ins.append((ins[j][0], push(sig) + push(pk), ins[j][2]))
                wit.append([])
                inputs.append((t, j, p2pkh(h), value))
            q += 1
        out_txs.append(serialize(version, new_ins, outs, wit, lock))
    return out_txs, inputs


def make_p2pkh_block(verifier, torch, n_tx: int = 2000, seed: int = P2PKH_SEED
                     ) -> Tuple[List[bytes], List[Tuple[int, int, bytes, int]]]:
    """BASELINE configs[0]: n_tx txs x 2 P2PKH inputs x 2 P2PKH outputs."""
    return make_block(verifier, torch, n_tx=n_tx, seed=seed, n_keys=4096, p2wpkh_share=0.0, inputs_per_tx=(2,))


class DeviceBlock:
    """A tx batch + its input jobs resident in HBM (struct hkv_txs with
    device pointers), for hkv_*_device calls."""

    def __init__(self, torch, txs: List[bytes], inputs: List[Tuple[int, int, bytes, int]]):
        from .lib import HkvTxs
        from .sighash import INPUT_JOB_DTYPE, TxBatch
        tb = TxBatch(txs)
        arr = np.zeros(len(inputs), dtype=INPUT_JOB_DTYPE)
        for k, (t, i, spk, value) in enumerate(inputs):
            off, ln = tb.script(spk)
            arr[k] = (t, i, off, ln, value)
        _, pool = tb.struct()

        def up(a):
            return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()

        self.d_bytes, self.d_off, self.d_pool, self.d_jobs = up(tb.bytes), up(tb.offsets), up(pool), up(arr)
        self.n = len(inputs)
        self.n_tx = len(txs)
        self.txs = HkvTxs(self.d_bytes.data_ptr(), self.d_off.data_ptr(), len(txs), self.d_pool.data_ptr(), tb._len)
        self.records = torch.zeros(max(1, self.n) * 168, dtype=torch.uint8, device="cuda")
        self.bits = torch.zeros((self.n + 63) // 64 * 2 + 2, dtype=torch.int32, device="cuda")


MULTISIG_SEED = 0x484B5643

# RIPEMD-160 for the P2SH script hashes of the generator (hashlib's is absent
# where OpenSSL 3 leaves it to the legacy provider): the published algorithm
# (Dobbertin, Bosselaers, Preneel 1996), message schedule and shifts below.
_RL = [list(range(16)), [7, 4, 13, 1, 10, 6, 15, 3, 12, 0, 9, 5, 2, 14, 11, 8],
       [3, 10, 14, 4, 9, 15, 8, 1, 2, 7, 0, 6, 13, 11, 5, 12], [1, 9, 11, 10, 0, 8, 12, 4, 13, 3, 7, 15, 14, 5, 6, 2],
       [4, 0, 5, 9, 7, 12, 2, 10, 14, 1, 3, 8, 11, 6, 15, 13]]
_RR = [[5, 14, 7, 0, 9, 2, 11, 4, 13, 6, 15, 8, 1, 10, 3, 12], [6, 11, 3, 7, 0, 13, 5, 10, 14, 15, 8, 12, 4, 9, 1, 2],
       [15, 5, 1, 3, 7, 14, 6, 9, 11, 8, 12, 2, 10, 0, 4, 13], [8, 6, 4, 1, 3, 11, 15, 0, 5, 12, 2, 13, 9, 7, 10, 14],
       [12, 15, 10, 4, 1, 5, 8, 7, 6, 2, 13, 14, 0, 3, 9, 11]]
_SL = [[11, 14, 15, 12, 5, 8, 7, 9, 11, 13, 14, 15, 6, 7, 9, 8], [7, 6, 8, 13, 11, 9, 7, 15, 7, 12, 15, 9, 11, 7, 13, 12],
       [11, 13, 6, 7, 14, 9, 13, 15, 14, 8, 13, 6, 5, 12, 7, 5], [11, 12, 14, 15, 14, 15, 9, 8, 9, 14, 5, 6, 8, 6, 5, 12],
       [9, 15, 5, 11, 6, 8, 13, 12, 5, 12, 13, 14, 11, 8, 5, 6]]
_SR = [[8, 9, 9, 11, 13, 15, 15, 5, 7, 7, 8, 11, 14, 14, 12, 6], [9, 13, 15, 7, 12, 8, 9, 11, 7, 7, 12, 7, 6, 15, 13, 11],
       [9, 7, 15, 11, 8, 6, 6, 14, 12, 13, 5, 14, 13, 13, 7, 5], [15, 5, 8, 11, 14, 14, 6, 14, 6, 9, 12, 9, 12, 5, 15, 8],
       [8, 5, 12, 9, 12, 5, 14, 6, 8, 13, 6, 5, 15, 13, 11, 11]]
_KL = [0, 0x5A827999, 0x6ED9EBA1, 0x8F1BBCDC, 0xA953FD4E]
_KR = [0x50A28BE6, 0x5C4DD124, 0x6D703EF3, 0x7A6D76E9, 0]


def _rmd_f(j, x, y, z):
    return [x ^ y ^ z, (x & y) | (~x & z), (x | ~y) ^ z, (x & z) | (y & ~z), x ^ (y | ~z)][j] & 0xFFFFFFFF


def ripemd160(data: bytes) -> bytes:
    rol = lambda x, n: ((x << n) | (x >> (32 - n))) & 0xFFFFFFFF  # noqa: E731
    h = [0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0]
    msg = data + b"\x80" + b"\0" * ((55 - len(data)) % 64) + struct.pack("<Q", 8 * len(data))
    for o in range(0, len(msg), 64):
        x = struct.unpack("<16I", msg[o:o + 64])
        al, bl, cl, dl, el = h
        ar, br, cr, dr, er = h
        for j in range(5):
            for i in range(16):
                t = rol((al + _rmd_f(j, bl, cl, dl) + x[_RL[j][i]] + _KL[j]) & 0xFFFFFFFF, _SL[j][i]) + el
                al, bl, cl, dl, el = el, t & 0xFFFFFFFF, bl, rol(cl, 10), dl
                t = rol((ar + _rmd_f(4 - j, br, cr, dr) + x[_RR[j][i]] + _KR[j]) & 0xFFFFFFFF, _SR[j][i]) + er
                ar, br, cr, dr, er = er, t & 0xFFFFFFFF, br, rol(cr, 10), dr
        h = [(h[1] + cl + dr) & 0xFFFFFFFF, (h[2] + dl + er) & 0xFFFFFFFF, (h[3] + el + ar) & 0xFFFFFFFF,
             (h[4] + al + br) & 0xFFFFFFFF, (h[0] + bl + cr) & 0xFFFFFFFF]
    return struct.pack("<5I", *h)


def multisig_script(m: int, pubs: List[bytes]) -> bytes:
    return bytes([0x50 + m]) + b"".join(push(p) for p in pubs) + bytes([0x50 + len(pubs), 0xAE])


def make_multisig_block(verifier, torch, n_tx: int, seed: int = MULTISIG_SEED, n_keys: int = 4096,
                        shapes=((1, 1), (1, 2), (2, 2), (2, 3), (1, 3), (3, 3)),
                        wraps=("p2sh", "bare", "p2wsh", "p2sh_p2wsh"), invalid_permille: int = 80
                        ) -> Tuple[List[bytes], List[Tuple[int, int, bytes, int]]]:
    """n_tx txs of one CHECKMULTISIG input each (m-of-n over compressed keys
    from a device-generated pool, bare or behind P2SH / P2WSH / P2SH-P2WSH,
    SIGHASH_ALL, no fork id): the multisig tail's workload at chunk scale.
    The sighash (legacy over the script for bare / P2SH, BIP143 over the
    witness script otherwise) comes from hkv_sighash, the signatures from
    hkv_gen_sign_device. About invalid_permille / 1000 of the inputs are
    damaged — a signer's signature made with another key, or two signatures
    swapped (m >= 2), or one signature dropped — so some verdicts reject.
    Returns (txs, inputs) as make_block does; the verdicts are the oracle's
    to decide (tests/test_gpu_ms_window.py)."""
    import hashlib
    rng = random.Random(seed)
    priv = torch.zeros(n_keys * 32, dtype=torch.uint8, device="cuda")
    pub = torch.zeros(n_keys * 33, dtype=torch.uint8, device="cuda")
    h160 = torch.zeros(n_keys * 20, dtype=torch.uint8, device="cuda")
    verifier.gen_keys_device(0, seed, n_keys, priv.data_ptr(), pub.data_ptr(), h160.data_ptr())
    torch.cuda.synchronize()
    pubs = pub.cpu().numpy().tobytes()
    metas, skel, hjobs = [], [], []
    for t in range(n_tx):
        m, n = rng.choice(shapes)
        wrap = rng.choice(wraps)
        kidx = rng.sample(range(n_keys), n)
        script = multisig_script(m, [pubs[33 * k:33 * k + 33] for k in kidx])
        wprog = b"\x00\x20" + hashlib.sha256(script).digest()
        h20 = lambda b: ripemd160(hashlib.sha256(b).digest())  # noqa: E731
        prev = {"bare": script, "p2sh": b"\xa9\x14" + h20(script) + b"\x87", "p2wsh": wprog,
                "p2sh_p2wsh": b"\xa9\x14" + h20(wprog) + b"\x87"}[wrap]
        value = rng.randrange(1000, 2**45)
        signers = sorted(rng.sample(range(n), m))
        damage = rng.randrange(1000) < invalid_permille
        kind = rng.choice(["wrong_key", "swap", "drop"]) if damage else None
        if kind == "swap" and m < 2:
            kind = "wrong_key"
        sign_keys = [kidx[j] for j in signers]
        if kind == "wrong_key":
            sign_keys[-1] = (sign_keys[-1] + 1 + rng.randrange(n_keys - 1)) % n_keys
        ins = [(rng.randbytes(32) + struct.pack("<I", rng.randrange(4)), b"", 0xFFFFFFFF)]
        outs = [(rng.randrange(546, 2**40), p2pkh(rng.randbytes(20))) for _ in range(2)]
        version, lock = rng.choice([1, 2]), rng.randrange(800000)
        skel.append(serialize(version, ins, outs, [], lock))
        seg = wrap in ("p2wsh", "p2sh_p2wsh")
        hjobs.append((t, 0, script, value, 1, HKV_SIGHASH_FORKID if seg else HKV_SIGHASH_LEGACY))
        metas.append((version, ins, outs, lock, script, wprog, prev, value, wrap, sign_keys, kind))
    msgs, status = tx_sig_hash_batch(verifier, skel, hjobs)
    assert not any(status), "skeleton txs must parse"
    sig_msgs, sig_keys = [], []
    for t, meta in enumerate(metas):
        for k in meta[9]:
            sig_msgs.append(msgs[t])
            sig_keys.append(k)
    d_msg = torch.from_numpy(np.frombuffer(b"".join(sig_msgs), dtype=np.uint8).copy()).cuda()
    d_idx = torch.tensor(sig_keys, dtype=torch.int32, device="cuda")
    d_sig = torch.zeros(len(sig_keys) * 64, dtype=torch.uint8, device="cuda")
    verifier.gen_sign_device(0, seed ^ 0x5167, len(sig_keys), priv.data_ptr(), d_idx.data_ptr(), d_msg.data_ptr(),
                             32, d_sig.data_ptr())
    torch.cuda.synchronize()
    sigs = d_sig.cpu().numpy().tobytes()
    out_txs, inputs, q = [], [], 0
    for t, (version, ins, outs, lock, script, wprog, prev, value, wrap, sign_keys, kind) in enumerate(metas):
        items = []
        for _ in sign_keys:
            items.append(der(sigs[64 * q:64 * q + 32], sigs[64 * q + 32:64 * q + 64]) + b"\x01")
            q += 1
        if kind == "swap":
            items[0], items[1] = items[1], items[0]
        elif kind == "drop":
            items = items[:-1]
        if wrap in ("p2wsh", "p2sh_p2wsh"):
            wit = [[b""] + items + [script]]
            ss = push(wprog) if wrap == "p2sh_p2wsh" else b""
        else:
            wit = [[]]
            ss = b"\x00" + b"".join(push(x) for x in items) + (push(script) if wrap == "p2sh" else b"")
        out_txs.append(serialize(version, [(ins[0][0], ss, ins[0][2])], outs, wit, lock))
        inputs.append((t, 0, prev, value))
    return out_txs, inputs
