"""Shared test setup. GPU tests are marked ``@pytest.mark.gpu`` and run only
on the MI355X box (``pytest -m gpu``); everything else runs on CPU."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "haskoin-node_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "libhkv_oracle.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


@pytest.fixture(scope="session")
def kat():
    """Golden KAT records + manifest (tests/golden/make_golden.py)."""
    with open(os.path.join(GOLDEN, "kat_manifest.json")) as f:
        man = json.load(f)
    data = open(os.path.join(GOLDEN, "kat_records.bin"), "rb").read()
    assert len(data) == man["count"] * man["record_size"]
    recs = [data[i * 168:(i + 1) * 168] for i in range(man["count"])]
    return recs, man["records"]


@pytest.fixture(scope="session")
def coracle():
    """The C restatement (oracle/hkv_oracle.c), built by __graft_entry__.build()."""
    import ctypes
    if not os.path.exists(ORACLE_SO):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                       stdout=subprocess.DEVNULL)
    lib = ctypes.CDLL(ORACLE_SO)
    lib.hkvo_verify_batch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_int]
    lib.hkvo_verify_record.argtypes = [ctypes.c_char_p, ctypes.c_int]
    lib.hkvo_pubkey_parse.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    return lib


OPENSSL_SO = os.path.join(ROOT, "oracle", "build", "libhkv_openssl.so")


@pytest.fixture(scope="session")
def openssl():
    """OpenSSL 3 ECDSA_do_verify behind the semantic adapter
    (oracle/openssl_check.c): an implementation-independent checker."""
    import ctypes
    if not os.path.exists(OPENSSL_SO):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                       stdout=subprocess.DEVNULL)
    lib = ctypes.CDLL(OPENSSL_SO)
    lib.hkvo_openssl_verify_batch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                              ctypes.c_void_p, ctypes.c_int]
    lib.hkvo_openssl_verify_batch.restype = ctypes.c_int
    return lib


def openssl_batch(lib, recs_bytes: bytes, mode: int, threads: int = 8):
    import ctypes
    import numpy as np
    n = len(recs_bytes) // 168
    out = np.zeros(n, dtype=np.uint8)
    buf = np.frombuffer(recs_bytes, dtype=np.uint8)
    rc = lib.hkvo_openssl_verify_batch(buf.ctypes.data_as(ctypes.c_void_p), n, mode,
                                       out.ctypes.data_as(ctypes.c_void_p), threads)
    assert rc == 0, "OpenSSL could not build a secp256k1 key"
    return out.astype(bool)


def host_threads() -> int:
    """Worker threads for the CPU checkers: this process's CPU share (the GPU
    box gives a job 16 CPUs even where os.cpu_count() shows the whole host)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", "16") or 16), 16))


def c_gen_batch(lib, seed: int, index0: int, n: int, npool: int, unc_permille: int, invalid_permille: int):
    """Records [index0, index0 + n) of the synthetic batch `seed` from the C
    restatement of the device generator (oracle/hkv_oracle.c hkvo_gen_batch):
    (records uint8[n*168], labels bool[n], classes int8[n], -1 = valid)."""
    import ctypes
    import numpy as np
    lib.hkvo_gen_batch.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_uint32,
                                   ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p]
    recs = np.zeros(n * 168, dtype=np.uint8)
    lab = np.zeros(n, dtype=np.uint8)
    cls = np.zeros(n, dtype=np.int8)
    rc = lib.hkvo_gen_batch(seed, index0, n, npool, unc_permille, invalid_permille, recs.ctypes.data,
                            lab.ctypes.data, cls.ctypes.data)
    assert rc == 0
    return recs, lab.astype(bool), cls


FAST_SO = os.path.join(ROOT, "oracle", "build", "libhkv_secpfast.so")


@pytest.fixture(scope="session")
def secpfast():
    """The libsecp256k1-class restatement (oracle/secp_fast.c): GLV + wNAF,
    5 x 52-bit field, safegcd — an algorithm independent of hkv_oracle.c's,
    and ~8x faster, so it can check every record of a 16M batch."""
    import ctypes
    if not os.path.exists(FAST_SO):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, stdout=subprocess.DEVNULL)
    lib = ctypes.CDLL(FAST_SO)
    lib.hkvo_fast_verify_batch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_int]
    return lib


def fast_batch(lib, recs, mode: int, threads: int = 8):
    import numpy as np
    recs = np.ascontiguousarray(np.frombuffer(bytes(recs), dtype=np.uint8) if isinstance(recs, bytes) else recs)
    n = len(recs) // 168
    out = np.zeros(n, dtype=np.uint8)
    lib.hkvo_fast_verify_batch(recs.ctypes.data, n, mode, out.ctypes.data, threads)
    return out.astype(bool)


def oracle_batch(lib, recs_bytes: bytes, mode: int, threads: int = 8):
    import ctypes
    import numpy as np
    n = len(recs_bytes) // 168
    out = np.zeros(n, dtype=np.uint8)
    buf = np.frombuffer(recs_bytes, dtype=np.uint8)
    lib.hkvo_verify_batch(buf.ctypes.data_as(ctypes.c_void_p), n, mode,
                          out.ctypes.data_as(ctypes.c_void_p), threads)
    return out.astype(bool)
