"""Batch verifier — the host-side mirror of the Haskell API the drop-in keeps.

Reference API (haskoin-core, un-vendored, pinned /root/reference/stack.yaml:10):
    verifyHashSig :: Ctx -> Hash256 -> Sig -> PubKey -> Bool
Batch equivalents, same per-element result:
    verify_hash_sig_batch(verifier, [(hash32, sig64, pubkey)]) -> [bool]   (HASKOIN)
    verify_raw_batch(verifier, [(msg32, sig64, pubkey)], mode)  -> [bool]
Errors follow the ABI: a verdict is never an error; a device failure raises
``HkvError`` (the Haskell wrapper maps it to an exception).
"""
from __future__ import annotations

import ctypes
import sys
from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from .lib import HKV_HASKOIN, HKV_LIBSECP, HKV_RECORD_SIZE, check, load_library
from .records import pack_records, unpack_bits


@dataclass
class VerifierConfig:
    """Mirrors the VerifierConfig record of the Haskell module."""
    device_ids: Optional[Sequence[int]] = None  # None: all visible devices
    flags: int = 0


class Verifier:
    """Owns one hkv_ctx (``withVerifier`` in the Haskell binding)."""

    def __init__(self, config: VerifierConfig | None = None):
        self.lib = load_library()
        # PyTorch-ROCm bundles its own HIP runtime; if libhkv's runtime (from
        # /opt/rocm) claims the device first, torch's later init finds no GPU.
        # When the caller already uses torch, initialise it first.
        tmod = sys.modules.get("torch")
        if tmod is not None:
            try:
                tmod.cuda.init()
            except Exception:  # pragma: no cover - no GPU / CPU-only torch
                pass
        self.config = config or VerifierConfig()
        ctx = ctypes.c_void_p()
        if self.config.device_ids is None:
            rc = self.lib.hkv_open(0, self.config.flags, ctypes.byref(ctx))
        else:
            ids = (ctypes.c_int * len(self.config.device_ids))(*self.config.device_ids)
            rc = self.lib.hkv_open_devices(ids, len(self.config.device_ids), self.config.flags,
                                           ctypes.byref(ctx))
        check(rc, "hkv_open", self.lib)
        self.ctx = ctx

    def close(self) -> None:
        if getattr(self, "ctx", None):
            self.lib.hkv_close(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    @property
    def num_devices(self) -> int:
        return self.lib.hkv_ctx_num_devices(self.ctx)

    # -- host-memory records --------------------------------------------------
    def verify_records(self, records: np.ndarray, mode: int) -> np.ndarray:
        """records: uint8 [n, 168] (or flat bytes) -> bool[n]."""
        arr = np.ascontiguousarray(np.asarray(records, dtype=np.uint8).reshape(-1))
        if arr.size % HKV_RECORD_SIZE:
            raise ValueError("record buffer is not a multiple of 168 bytes")
        n = arr.size // HKV_RECORD_SIZE
        words = np.zeros(max(1, (n + 31) // 32), dtype=np.uint32)
        if n:
            rc = self.lib.hkv_verify_host(self.ctx, arr.ctypes.data_as(ctypes.c_void_p), n, mode,
                                          words.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
            check(rc, "hkv_verify_host", self.lib)
        return unpack_bits(words, n)

    # -- device-resident records (torch tensors on this rank's GPU) ----------
    def verify_device(self, dev: int, d_records_ptr: int, n: int, mode: int, d_bits_ptr: int,
                      stream_ptr: int = 0) -> None:
        rc = self.lib.hkv_verify_device(self.ctx, dev, ctypes.c_void_p(d_records_ptr), n, mode,
                                        ctypes.c_void_p(d_bits_ptr), ctypes.c_void_p(stream_ptr or None))
        check(rc, "hkv_verify_device", self.lib)

    def gen_records_device(self, dev: int, seed: int, n: int, pool_size: int, unc_permille: int,
                           d_records_ptr: int, stream_ptr: int = 0) -> None:
        rc = self.lib.hkv_gen_records_device(self.ctx, dev, seed, n, pool_size, unc_permille,
                                             ctypes.c_void_p(d_records_ptr),
                                             ctypes.c_void_p(stream_ptr or None))
        check(rc, "hkv_gen_records_device", self.lib)

    def gen_batch_device(self, dev: int, seed: int, index0: int, n: int, pool_size: int, unc_permille: int,
                         invalid_permille: int, d_records_ptr: int, d_labels_ptr: int = 0,
                         stream_ptr: int = 0) -> None:
        """Records [index0, index0 + n) of the synthetic batch `seed`
        (hkv_gen_batch_device), with construction labels when d_labels_ptr."""
        rc = self.lib.hkv_gen_batch_device(self.ctx, dev, seed, index0, n, pool_size, unc_permille, invalid_permille,
                                           ctypes.c_void_p(d_records_ptr), ctypes.c_void_p(d_labels_ptr or None),
                                           ctypes.c_void_p(stream_ptr or None))
        check(rc, "hkv_gen_batch_device", self.lib)

    # -- signature hashes / standard inputs on device (hkv_*_device) ---------
    def sighash_device(self, dev: int, d_txs, d_jobs: int, n: int, forkid: int, d_out: int, out_stride: int,
                       d_status: int = 0, stream_ptr: int = 0) -> None:
        rc = self.lib.hkv_sighash_device(self.ctx, dev, ctypes.byref(d_txs), ctypes.c_void_p(d_jobs), n, forkid,
                                         ctypes.c_void_p(d_out), out_stride, ctypes.c_void_p(d_status or None),
                                         ctypes.c_void_p(stream_ptr or None))
        check(rc, "hkv_sighash_device", self.lib)

    def std_inputs_device(self, dev: int, d_txs, d_jobs: int, n: int, forkid: int, d_records: int,
                          stream_ptr: int = 0) -> None:
        rc = self.lib.hkv_std_inputs_device(self.ctx, dev, ctypes.byref(d_txs), ctypes.c_void_p(d_jobs), n, forkid,
                                            ctypes.c_void_p(d_records), ctypes.c_void_p(stream_ptr or None))
        check(rc, "hkv_std_inputs_device", self.lib)

    def verify_std_inputs_device(self, dev: int, d_txs, d_jobs: int, n: int, forkid: int, d_records: int,
                                 d_bits: int, stream_ptr: int = 0, d_status: int = 0) -> None:
        """hkv_verify_std_inputs_device, or with d_status (a device word the
        caller zeroed) hkv_verify_std_inputs_device_status."""
        if d_status:
            rc = self.lib.hkv_verify_std_inputs_device_status(
                self.ctx, dev, ctypes.byref(d_txs), ctypes.c_void_p(d_jobs), n, forkid, ctypes.c_void_p(d_records),
                ctypes.c_void_p(d_bits), ctypes.c_void_p(d_status), ctypes.c_void_p(stream_ptr or None))
            check(rc, "hkv_verify_std_inputs_device_status", self.lib)
            return
        rc = self.lib.hkv_verify_std_inputs_device(self.ctx, dev, ctypes.byref(d_txs), ctypes.c_void_p(d_jobs), n,
                                                   forkid, ctypes.c_void_p(d_records), ctypes.c_void_p(d_bits),
                                                   ctypes.c_void_p(stream_ptr or None))
        check(rc, "hkv_verify_std_inputs_device", self.lib)

    def device_fault(self, dev: int) -> int:
        """hkv_device_fault: read and clear device dev's sticky fault latch."""
        w = ctypes.c_uint32(0)
        check(self.lib.hkv_device_fault(self.ctx, dev, ctypes.byref(w)), "hkv_device_fault", self.lib)
        return w.value

    def gen_keys_device(self, dev: int, seed: int, n: int, d_priv: int, d_pub: int, d_h160: int,
                        stream_ptr: int = 0) -> None:
        rc = self.lib.hkv_gen_keys_device(self.ctx, dev, seed, n, ctypes.c_void_p(d_priv), ctypes.c_void_p(d_pub),
                                          ctypes.c_void_p(d_h160), ctypes.c_void_p(stream_ptr or None))
        check(rc, "hkv_gen_keys_device", self.lib)

    def gen_sign_device(self, dev: int, seed: int, n: int, d_priv: int, d_key_idx: int, d_msg: int, msg_stride: int,
                        d_sig: int, stream_ptr: int = 0) -> None:
        rc = self.lib.hkv_gen_sign_device(self.ctx, dev, seed, n, ctypes.c_void_p(d_priv),
                                          ctypes.c_void_p(d_key_idx or None), ctypes.c_void_p(d_msg), msg_stride,
                                          ctypes.c_void_p(d_sig), ctypes.c_void_p(stream_ptr or None))
        check(rc, "hkv_gen_sign_device", self.lib)

    def debug_op(self, dev: int, op: int, n: int, d_a: int, d_b: int, d_out: int, stream_ptr: int = 0) -> None:
        rc = self.lib.hkv_debug_op(self.ctx, dev, op, n, ctypes.c_void_p(d_a), ctypes.c_void_p(d_b),
                                   ctypes.c_void_p(d_out), ctypes.c_void_p(stream_ptr or None))
        check(rc, "hkv_debug_op", self.lib)


def verify_raw_batch(verifier: Verifier, items: Iterable[Tuple[bytes, bytes, bytes]],
                     mode: int = HKV_LIBSECP) -> List[bool]:
    """(msg32, compact sig r||s, SEC1 pubkey bytes) -> verdicts; mode
    HKV_LIBSECP = secp256k1_ecdsa_verify, HKV_HASKOIN = verifyHashSig."""
    recs = pack_records(items)
    return verifier.verify_records(recs, mode).tolist()


def verify_hash_sig_batch(verifier: Verifier, items: Iterable[Tuple[bytes, bytes, bytes]]) -> List[bool]:
    """Batch ``verifyHashSig``: element i equals verifyHashSig ctx h_i sig_i pub_i."""
    return verify_raw_batch(verifier, items, HKV_HASKOIN)
