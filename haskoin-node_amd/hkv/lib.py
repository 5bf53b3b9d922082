"""ctypes binding of libhkv.so (include/hkv.h). One definition per exported
symbol, mirroring the header; ``EXPORTS`` is checked against the header by
``tests/test_abi.py``."""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_int, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p

HKV_RECORD_SIZE = 168
HKV_LIBSECP = 0
HKV_HASKOIN = 1

HKV_SIGHASH_LEGACY = 0
HKV_SIGHASH_FORKID = 1
HKV_NO_FORKID = -1
HKV_SH_OK, HKV_SH_BAD_TX, HKV_SH_BAD_INPUT, HKV_SH_BAD_REF = 0, 1, 2, 3

HKV_HDR_POW_OK, HKV_HDR_LINK_OK, HKV_HDR_NEGATIVE, HKV_HDR_OVERFLOW = 0x01, 0x02, 0x04, 0x08
HKV_HDR_ZERO_TARGET, HKV_HDR_ABOVE_LIMIT, HKV_HDR_HASH_ABOVE = 0x10, 0x20, 0x40

HKV_OK = 0
HKV_FAIL_NONE, HKV_FAIL_ENQUEUE, HKV_FAIL_JOIN, HKV_FAIL_ALLOC, HKV_FAIL_TAIL = 0, 1, 2, 3, 4
HKV_STATUS_TAIL_FAULT = 1
_ERRS = {-1: "HKV_E_ARG", -2: "HKV_E_NODEV", -3: "HKV_E_OOM", -4: "HKV_E_HIP", -5: "HKV_E_INTERNAL"}

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def lib_path() -> str:
    return os.environ.get("HKV_LIB", os.path.join(_PKG_DIR, "lib", "libhkv.so"))


class HkvError(RuntimeError):
    def __init__(self, rc: int, what: str, lib=None):
        detail = ""
        if lib is not None:
            try:
                detail = lib.hkv_last_hip_error().decode()
            except Exception:  # pragma: no cover - best effort
                detail = ""
        super().__init__(f"{what}: {_ERRS.get(rc, rc)} {detail}".strip())
        self.rc = rc


class HkvTxs(ctypes.Structure):
    """struct hkv_txs (include/hkv.h)."""
    _fields_ = [("bytes", c_void_p), ("offsets", c_void_p), ("n_tx", c_uint32), ("scripts", c_void_p),
                ("scripts_len", c_uint32)]


class HkvSighashJob(ctypes.Structure):
    _fields_ = [("tx", c_uint32), ("input", c_uint32), ("script_off", c_uint32), ("script_len", c_uint32),
                ("value", c_uint64), ("sighash", c_uint32), ("kind", c_uint32)]


class HkvInputJob(ctypes.Structure):
    _fields_ = [("tx", c_uint32), ("input", c_uint32), ("script_off", c_uint32), ("script_len", c_uint32),
                ("value", c_uint64)]


assert ctypes.sizeof(HkvSighashJob) == 32 and ctypes.sizeof(HkvInputJob) == 24

# name -> (restype, argtypes)
EXPORTS = {
    "hkv_open": (c_int, [c_int, c_uint32, POINTER(c_void_p)]),
    "hkv_open_devices": (c_int, [POINTER(c_int), c_int, c_uint32, POINTER(c_void_p)]),
    "hkv_close": (None, [c_void_p]),
    "hkv_ctx_num_devices": (c_int, [c_void_p]),
    "hkv_device_healthy": (c_int, [c_void_p, c_int]),
    "hkv_device_failures": (c_int, [c_void_p, c_int]),
    "hkv_device_reset_health": (c_int, [c_void_p, c_int]),
    "hkv_debug_fail_device": (c_int, [c_void_p, c_int, c_uint32]),
    "hkv_debug_ms_window": (c_int, [c_void_p, c_int, c_uint32, c_uint32]),
    "hkv_debug_ms_scratch": (c_int, [c_void_p, c_int, POINTER(c_size_t)]),
    "hkv_batch_alloc": (c_int, [c_void_p, c_size_t, POINTER(c_void_p)]),
    "hkv_batch_free": (None, [c_void_p]),
    "hkv_batch_records": (POINTER(c_uint8), [c_void_p]),
    "hkv_batch_capacity": (c_size_t, [c_void_p]),
    "hkv_verify": (c_int, [c_void_p, c_void_p, c_size_t, c_uint32, POINTER(c_uint32)]),
    "hkv_verify_host": (c_int, [c_void_p, c_void_p, c_size_t, c_uint32, POINTER(c_uint32)]),
    "hkv_verify_device": (c_int, [c_void_p, c_int, c_void_p, c_size_t, c_uint32, c_void_p, c_void_p]),
    "hkv_gen_records_device": (c_int, [c_void_p, c_int, c_uint64, c_size_t, c_uint32, c_uint32, c_void_p,
                                       c_void_p]),
    "hkv_gen_batch_device": (c_int, [c_void_p, c_int, c_uint64, c_uint64, c_size_t, c_uint32, c_uint32, c_uint32,
                                     c_void_p, c_void_p, c_void_p]),
    "hkv_sighash": (c_int, [c_void_p, POINTER(HkvTxs), c_void_p, c_size_t, ctypes.c_int32, c_void_p, c_void_p]),
    "hkv_sighash_device": (c_int, [c_void_p, c_int, POINTER(HkvTxs), c_void_p, c_size_t, ctypes.c_int32, c_void_p,
                                   c_size_t, c_void_p, c_void_p]),
    "hkv_std_inputs_device": (c_int, [c_void_p, c_int, POINTER(HkvTxs), c_void_p, c_size_t, ctypes.c_int32,
                                      c_void_p, c_void_p]),
    "hkv_verify_std_inputs_device": (c_int, [c_void_p, c_int, POINTER(HkvTxs), c_void_p, c_size_t, ctypes.c_int32,
                                             c_void_p, c_void_p, c_void_p]),
    "hkv_verify_std_inputs_device_status": (c_int, [c_void_p, c_int, POINTER(HkvTxs), c_void_p, c_size_t,
                                                    ctypes.c_int32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "hkv_device_fault": (c_int, [c_void_p, c_int, POINTER(c_uint32)]),
    "hkv_verify_std_inputs": (c_int, [c_void_p, POINTER(HkvTxs), c_void_p, c_size_t, ctypes.c_int32,
                                      POINTER(c_uint32)]),
    "hkv_merkle_roots": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p]),
    "hkv_merkle_roots_device": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p,
                                        c_void_p]),
    "hkv_check_headers": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p]),
    "hkv_check_headers_device": (c_int, [c_void_p, c_int, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p]),
    "hkv_gen_keys_device": (c_int, [c_void_p, c_int, c_uint64, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p]),
    "hkv_gen_sign_device": (c_int, [c_void_p, c_int, c_uint64, c_size_t, c_void_p, c_void_p, c_void_p, c_size_t,
                                    c_void_p, c_void_p]),
    "hkv_debug_op": (c_int, [c_void_p, c_int, c_uint32, c_size_t, c_void_p, c_void_p, c_void_p, c_void_p]),
    "hkv_profile_enable": (c_int, [c_void_p, c_int]),
    "hkv_profile_read": (c_int, [c_void_p, c_int, POINTER(ctypes.c_double), POINTER(ctypes.c_double),
                                 POINTER(c_uint64)]),
    "hkv_profile_clock": (c_int, [c_void_p, c_int, POINTER(ctypes.c_double)]),
    "hkv_profile_phases": (c_int, [c_void_p, c_int, POINTER(c_uint64), c_size_t, POINTER(ctypes.c_double)]),
    "hkv_profile_group_stamps": (c_int, [c_void_p, c_int, POINTER(c_uint64), c_size_t, POINTER(ctypes.c_double)]),
    "hkv_strerror": (c_char_p, [c_int]),
    "hkv_last_hip_error": (c_char_p, []),
    "hkv_device_count": (c_int, []),
    "hkv_version": (c_uint32, []),
}

# measurement hooks a library variant built before them may lack; every other
# export is required (tests/test_abi.py checks the in-tree build has them all)
MEASUREMENT_ONLY = {"hkv_profile_group_stamps"}

_LIB = None


def load_library(path: str | None = None):
    """Load libhkv.so and bind every export. Raises if the library is absent:
    the product path has no fallback."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or lib_path()
    if not os.path.exists(p):
        raise ImportError(f"libhkv.so not built at {p}; run __graft_entry__.build()")
    lib = ctypes.CDLL(p)
    for name, (res, args) in EXPORTS.items():
        if name in MEASUREMENT_ONLY and not hasattr(lib, name):
            continue  # (an older library loaded for a same-box A/B: HKV_LIB)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _LIB = lib
    return lib


def check(rc: int, what: str, lib=None) -> None:
    if rc != HKV_OK:
        raise HkvError(rc, what, lib)
