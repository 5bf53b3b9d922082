"""hkv — MI355X batch secp256k1 ECDSA verification (host side, ctypes over
the C ABI in ``include/hkv.h``).

This is the Python face of the product path; it loads the in-tree
``haskoin-node_amd/lib/libhkv.so`` (built by ``__graft_entry__.build()``)
and fails loudly when it is missing. There is no CPU fallback.
"""
from .lib import (HKV_HASKOIN, HKV_LIBSECP, HKV_NO_FORKID, HKV_RECORD_SIZE, HKV_SIGHASH_FORKID,
                  HKV_SIGHASH_LEGACY, HkvError, HkvTxs, lib_path, load_library)
from .records import make_record, pack_records, unpack_bits
from .headers import check_headers, check_headers_device
from .merkle import merkle_roots, merkle_roots_device
from .sighash import TxBatch, tx_sig_hash_batch, verify_std_inputs
from .verify import (Verifier, VerifierConfig, verify_hash_sig_batch,
                     verify_raw_batch)
from .actor import VerifyActor, VerifyActorConfig

__all__ = [
    "HKV_HASKOIN", "HKV_LIBSECP", "HKV_RECORD_SIZE", "HkvError", "lib_path",
    "load_library", "make_record", "pack_records", "unpack_bits", "Verifier",
    "VerifierConfig", "verify_hash_sig_batch", "verify_raw_batch", "HKV_NO_FORKID",
    "HKV_SIGHASH_FORKID", "HKV_SIGHASH_LEGACY", "HkvTxs", "TxBatch", "tx_sig_hash_batch",
    "verify_std_inputs", "check_headers", "check_headers_device",
    "merkle_roots", "merkle_roots_device", "VerifyActor", "VerifyActorConfig",
]
