"""CPU tests of the drop-in boundary: libhkv.so loads and exports exactly the
functions include/hkv.h declares (no compute calls — there is no GPU here)."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "hkv.h")
LIB = os.path.join(ROOT, "haskoin-node_amd", "lib", "libhkv.so")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(hkv_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "haskoin-node_amd", "csrc")], check=True,
                       stdout=subprocess.DEVNULL)
    import hkv
    return hkv.load_library()


def test_header_declares_expected_surface():
    names = header_functions()
    for required in ("hkv_open", "hkv_close", "hkv_batch_alloc", "hkv_batch_free", "hkv_batch_records",
                     "hkv_verify", "hkv_strerror"):
        assert required in names  # SURVEY.md §8(b) ABI


def test_library_exports_every_header_symbol(lib):
    import hkv.lib as hl
    names = header_functions()
    assert sorted(hl.EXPORTS) == names
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (hkv_\w+)", out))
    assert set(names) <= exported
    # nothing hkv_* exported beyond the header
    assert exported == set(names)


def test_error_strings_and_version(lib):
    assert lib.hkv_strerror(0) == b"ok"
    assert lib.hkv_strerror(-1) == b"invalid argument"
    assert lib.hkv_version() >> 16 == 1


def test_bad_arguments_rejected_without_device(lib):
    import ctypes
    assert lib.hkv_open(0, 0, None) == -1
    assert lib.hkv_verify(None, None, 0, 0, None) == -1
    assert lib.hkv_verify_device(None, 0, None, 0, 0, None, None) == -1
    assert lib.hkv_batch_alloc(None, 10, ctypes.byref(ctypes.c_void_p())) == -1
    assert lib.hkv_debug_ms_window(None, 0, 64, 64) == -1
    assert lib.hkv_debug_ms_scratch(None, 0, ctypes.byref(ctypes.c_size_t())) == -1
    assert lib.hkv_device_fault(None, 0, ctypes.byref(ctypes.c_uint32())) == -1


def test_kernel_code_object_is_gfx950():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", LIB], capture_output=True, text=True)
    # the offload bundle is embedded; check the target string is present in the binary
    blob = open(LIB, "rb").read()
    assert b"gfx950" in blob
    assert b"gfx942" not in blob and b"gfx90a" not in blob


def test_native_caller_builds_and_links_only_the_c_abi():
    """tools/native_latency (bench.py config0.native_caller) is built with the
    library and calls it through include/hkv.h alone: it links libhkv.so from
    the tree (rpath) and imports only hkv_* symbols from it; without a block
    directory it prints its usage and exits 2 before touching a device."""
    tool = os.path.join(ROOT, "tools", "native_latency")
    if not os.path.exists(tool):
        subprocess.run(["make", "-C", os.path.join(ROOT, "haskoin-node_amd", "csrc")], check=True,
                       stdout=subprocess.DEVNULL)
    ldd = subprocess.run(["ldd", tool], capture_output=True, text=True, check=True).stdout
    assert os.path.realpath(LIB) in {os.path.realpath(l.split("=>")[1].split("(")[0].strip())
                                     for l in ldd.splitlines() if "libhkv.so" in l}
    nm = subprocess.run(["nm", "-D", "--undefined-only", tool], capture_output=True, text=True, check=True).stdout
    used = sorted({l.split()[-1] for l in nm.splitlines() if l.split() and l.split()[-1].startswith("hkv_")})
    assert used and set(used) <= set(header_functions()), used
    p = subprocess.run([tool], capture_output=True, text=True)
    assert p.returncode == 2 and "usage" in p.stderr
