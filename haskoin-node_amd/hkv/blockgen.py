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
