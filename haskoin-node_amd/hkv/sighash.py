"""Batch signature hashes and standard-input verification — the host-side
mirror of the haskoin-core functions the drop-in keeps (SURVEY.md §8(a)
a7-a9, §8(f) row 2). All computation runs in libhkv's HIP kernels.

Reference API (haskoin-core-1.1.0, un-vendored, pinned
/root/reference/stack.yaml:10):

    txSigHash       :: Network -> Tx -> Script -> Word64 -> Int -> SigHash -> Hash256
    txSigHashForkId :: Network -> Tx -> Script -> Word64 -> Int -> SigHash -> Hash256
    verifyStdInput  :: Network -> Ctx -> Tx -> Int -> ScriptOutput -> Word64 -> Bool

Batch equivalents (same per-element result):

    tx_sig_hash_batch(v, txs, [(tx, input, script_code, value, sighash, kind)], forkid)
        -> [Hash256 bytes], [status]
    verify_std_inputs(v, txs, [(tx, input, prevout_script, value)], forkid) -> [bool]

``txs`` are serialised transactions (wire form; the BIP144 witness form is
accepted). ``forkid`` is None for a network without a fork id (BTC) or the
network's fork id (0 for BCH), like haskoin's ``getSigHashForkId net``.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .lib import (HKV_NO_FORKID, HKV_SIGHASH_FORKID, HKV_SIGHASH_LEGACY, HkvInputJob, HkvSighashJob, HkvTxs,
                  check)
from .records import unpack_bits

SIGHASH_JOB_DTYPE = np.dtype([("tx", "<u4"), ("input", "<u4"), ("script_off", "<u4"), ("script_len", "<u4"),
                              ("value", "<u8"), ("sighash", "<u4"), ("kind", "<u4")])
INPUT_JOB_DTYPE = np.dtype([("tx", "<u4"), ("input", "<u4"), ("script_off", "<u4"), ("script_len", "<u4"),
                            ("value", "<u8")])
assert SIGHASH_JOB_DTYPE.itemsize == ctypes.sizeof(HkvSighashJob)
assert INPUT_JOB_DTYPE.itemsize == ctypes.sizeof(HkvInputJob)


def _forkid(forkid: Optional[int]) -> int:
    return HKV_NO_FORKID if forkid is None else int(forkid)


class TxBatch:
    """Host-side tx batch: concatenated wire bytes, n_tx + 1 offsets and a
    deduplicated script pool (struct hkv_txs)."""

    def __init__(self, txs: Sequence[bytes]):
        self.offsets = np.zeros(len(txs) + 1, dtype=np.uint32)
        if txs:
            self.offsets[1:] = np.cumsum([len(t) for t in txs], dtype=np.uint64).astype(np.uint32)
        self.bytes = np.frombuffer(b"".join(txs) or b"\0", dtype=np.uint8).copy()
        self._scripts: List[bytes] = []
        self._where = {}
        self._len = 0

    def script(self, s: bytes) -> Tuple[int, int]:
        """(offset, length) of s in the script pool."""
        if s not in self._where:
            self._where[s] = self._len
            self._scripts.append(s)
            self._len += len(s)
        return self._where[s], len(s)

    def struct(self) -> Tuple[HkvTxs, np.ndarray]:
        pool = np.frombuffer(b"".join(self._scripts) or b"\0", dtype=np.uint8).copy()
        st = HkvTxs(self.bytes.ctypes.data, self.offsets.ctypes.data, len(self.offsets) - 1, pool.ctypes.data,
                    self._len)
        return st, pool  # keep pool alive while st is used


def tx_sig_hash_batch(verifier, txs: Sequence[bytes], jobs: Sequence[Tuple[int, int, bytes, int, int, int]],
                      forkid: Optional[int] = None) -> Tuple[List[bytes], List[int]]:
    """jobs: (tx index, input index, scriptCode bytes, value, sighash word,
    kind: HKV_SIGHASH_LEGACY (txSigHash) / HKV_SIGHASH_FORKID (txSigHashForkId)).
    Returns the 32-byte hashes and per-job status (HKV_SH_*)."""
    tb = TxBatch(txs)
    arr = np.zeros(len(jobs), dtype=SIGHASH_JOB_DTYPE)
    for k, (t, i, code, value, sh, kind) in enumerate(jobs):
        off, ln = tb.script(code)
        arr[k] = (t, i, off, ln, value, sh & 0xFFFFFFFF, kind)
    st, pool = tb.struct()
    out = np.zeros((max(1, len(jobs)), 32), dtype=np.uint8)
    status = np.zeros(max(1, len(jobs)), dtype=np.uint8)
    rc = verifier.lib.hkv_sighash(verifier.ctx, ctypes.byref(st), arr.ctypes.data, len(jobs), _forkid(forkid),
                                  out.ctypes.data, status.ctypes.data)
    check(rc, "hkv_sighash", verifier.lib)
    return [out[k].tobytes() for k in range(len(jobs))], [int(x) for x in status[:len(jobs)]]


def verify_std_inputs(verifier, txs: Sequence[bytes], inputs: Sequence[Tuple[int, int, bytes, int]],
                      forkid: Optional[int] = None) -> List[bool]:
    """Batch verifyStdInput: inputs = (tx index, input index, prevout
    scriptPubKey, prevout value); P2PK / P2PKH / P2WPKH prevouts."""
    tb = TxBatch(txs)
    arr = np.zeros(len(inputs), dtype=INPUT_JOB_DTYPE)
    for k, (t, i, spk, value) in enumerate(inputs):
        off, ln = tb.script(spk)
        arr[k] = (t, i, off, ln, value)
    st, pool = tb.struct()
    words = np.zeros(max(1, (len(inputs) + 31) // 32), dtype=np.uint32)
    rc = verifier.lib.hkv_verify_std_inputs(verifier.ctx, ctypes.byref(st), arr.ctypes.data, len(inputs),
                                            _forkid(forkid), words.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    check(rc, "hkv_verify_std_inputs", verifier.lib)
    return unpack_bits(words, len(inputs)).tolist()


__all__ = ["TxBatch", "tx_sig_hash_batch", "verify_std_inputs", "SIGHASH_JOB_DTYPE", "INPUT_JOB_DTYPE",
           "HKV_SIGHASH_LEGACY", "HKV_SIGHASH_FORKID"]
