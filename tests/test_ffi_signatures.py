"""The Haskell FFI against include/hkv.h, mechanically.

GHC is absent here, so the `foreign import ccall` bindings of
haskell/Haskoin/Node/Verify/FFI.hs and INTEGRATION.md are checked by parsing:
every bound symbol must be a prototype of include/hkv.h with the same arity,
the same C type per argument (CInt <-> int, CSize <-> size_t, Word32 <->
uint32_t, Int32 <-> int32_t, Word64 <-> uint64_t, CString <-> const char*,
Ptr a <-> a pointer whose pointee matches a, or void*) and the same result
(IO () <-> void). The binding replaces secp256k1-haskell's per-signature FFI
(/root/reference/stack.yaml:9). The checker itself is tested on deliberately
wrong bindings (an argument dropped, a CInt where the C side takes size_t)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hkv.h")
FFI_HS = os.path.join(ROOT, "haskell", "Haskoin", "Node", "Verify", "FFI.hs")
INTEGRATION = os.path.join(ROOT, "INTEGRATION.md")

# Haskell scalar type -> the C type it marshals to (Foreign.C.Types / Data.Word)
SCALARS = {"CInt": "int", "CUInt": "unsigned", "CSize": "size_t", "Word8": "uint8_t", "Word32": "uint32_t",
           "Int32": "int32_t", "Word64": "uint64_t", "Int64": "int64_t", "CDouble": "double", "Double": "double"}
# Haskell pointee -> the C pointee names it may stand for (void always allowed)
POINTEES = {"HkvCtx": {"hkv_ctx"}, "HkvBatch": {"hkv_batch"}, "HkvTxs": {"hkv_txs"},
            "InputJob": {"hkv_input_job"}, "SighashJob": {"hkv_sighash_job"}, "Word8": {"uint8_t"},
            "Word32": {"uint32_t"}, "Word64": {"uint64_t"}, "CInt": {"int"}, "CDouble": {"double"},
            "Double": {"double"}, "()": {"void"}, "CChar": {"char"}}


def c_prototypes(text: str) -> dict:
    """name -> (result type, [argument types]) for every prototype in hkv.h,
    each type normalised to (base name, pointer depth); const dropped."""
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    text = re.sub(r"#[^\n]*", " ", text)
    out = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(hkv_\w+)\s*\(([^;{}()]*)\)\s*;", text):
        ret, name, args = m.group(1), m.group(2), m.group(3).strip()
        if "typedef" in ret or "struct" in ret:
            continue
        params = [] if args in ("", "void") else [a.strip() for a in args.split(",")]
        out[name] = (_ctype(ret), [_ctype(re.sub(r"\s*\b\w+$", "", p) if not p.endswith("*") else p)
                                   for p in params])
    return out


def _ctype(s: str):
    s = " ".join(s.replace("const", " ").split())
    depth = s.count("*")
    base = s.replace("*", " ").split()
    base = " ".join(base) if base else ""
    return base, depth


def hs_bindings(text: str) -> dict:
    """symbol -> [(Haskell name, [argument types], result type)] for every
    `foreign import ccall [safe|unsafe] "sym" name :: T -> ... -> IO R` (the
    signature may span lines)."""
    out = {}
    pat = re.compile(r'foreign\s+import\s+ccall\s+(?:safe|unsafe)?\s*"([\w]+)"\s+(\w+)\s*::\s*(.*?)(?=\n\S|\n\s*\n|\n\s*--|\Z)',
                     re.S)
    for m in pat.finditer(text):
        sig = " ".join(re.sub(r"--[^\n]*", " ", m.group(3)).split())  # (trailing comments dropped)
        sym, name = m.group(1), m.group(2)
        parts = _split_arrows(sig)
        res = parts[-1]
        assert res.startswith("IO "), (sym, sig)
        out.setdefault(sym, []).append((name, parts[:-1], res[3:].strip()))
    return out


def _split_arrows(sig: str):
    parts, depth, cur = [], 0, ""
    i = 0
    while i < len(sig):
        c = sig[i]
        if c == "(":
            depth += 1
        elif c == ")":
            depth -= 1
        if depth == 0 and sig.startswith("->", i):
            parts.append(cur.strip())
            cur = ""
            i += 2
            continue
        cur += c
        i += 1
    parts.append(cur.strip())
    return parts


def _hs_matches(hs: str, c) -> bool:
    base, depth = c
    hs = hs.strip()
    while hs.startswith("(") and hs.endswith(")") and hs != "()":
        hs = hs[1:-1].strip()
    if hs == "()":
        return base == "void" and depth == 0
    if hs == "CString":
        return base == "char" and depth == 1
    if hs.startswith("Ptr ") or hs.startswith("FunPtr "):
        inner = hs.split(" ", 1)[1].strip()
        if depth < 1:
            return False
        if base == "void" and depth == 1:
            return True
        ip = inner
        while ip.startswith("(") and ip.endswith(")") and ip != "()":
            ip = ip[1:-1].strip()
        if ip.startswith("Ptr "):
            return _hs_matches(ip, (base, depth - 1))
        return depth == 1 and base in POINTEES.get(ip, set())
    return depth == 0 and SCALARS.get(hs) == base


def check_bindings(hs_text: str, protos: dict) -> list:
    """Every problem found (empty: the bindings match the header)."""
    errs = []
    for sym, binds in hs_bindings(hs_text).items():
        if sym not in protos:
            errs.append(f"{sym}: not declared in include/hkv.h")
            continue
        cres, cargs = protos[sym]
        for name, args, res in binds:
            if len(args) != len(cargs):
                errs.append(f"{sym} ({name}): arity {len(args)}, hkv.h has {len(cargs)}")
                continue
            for k, (h, c) in enumerate(zip(args, cargs)):
                if not _hs_matches(h, c):
                    errs.append(f"{sym} ({name}): argument {k + 1} is {h}, hkv.h has {c[0]}{'*' * c[1]}")
            if not _hs_matches(res, cres):
                errs.append(f"{sym} ({name}): result IO {res}, hkv.h returns {cres[0]}{'*' * cres[1]}")
    return errs


@pytest.fixture(scope="module")
def protos():
    return c_prototypes(open(HEADER).read())


def test_header_parses(protos):
    assert protos["hkv_verify_std_inputs_device_status"][1] == [
        ("hkv_ctx", 1), ("int", 0), ("hkv_txs", 1), ("hkv_input_job", 1), ("size_t", 0), ("int32_t", 0),
        ("void", 1), ("uint32_t", 1), ("uint32_t", 1), ("void", 1)]
    assert protos["hkv_close"] == (("void", 0), [("hkv_ctx", 1)])
    assert protos["hkv_open"][1][2] == ("hkv_ctx", 2)
    assert protos["hkv_strerror"][0] == ("char", 1)
    assert len(protos) >= 40


@pytest.mark.parametrize("path", [FFI_HS, INTEGRATION])
def test_ffi_bindings_match_header(protos, path):
    text = open(path).read()
    binds = hs_bindings(text)
    assert binds, f"no foreign import found in {path}"
    assert check_bindings(text, protos) == []


def test_ffi_binds_the_fault_reporting(protos):
    """The actor's error policy needs the status form and the latch."""
    binds = hs_bindings(open(FFI_HS).read())
    for sym in ("hkv_verify_std_inputs", "hkv_verify_std_inputs_device_status", "hkv_device_fault",
                "hkv_verify", "hkv_open", "hkv_close", "hkv_strerror"):
        assert sym in binds, sym


def test_checker_rejects_wrong_bindings(protos):
    good = open(FFI_HS).read()
    # an argument dropped
    bad = good.replace("c_hkv_device_fault :: Ptr HkvCtx -> CInt -> Ptr Word32 -> IO CInt",
                       "c_hkv_device_fault :: Ptr HkvCtx -> Ptr Word32 -> IO CInt")
    assert bad != good
    assert any("arity" in e and "hkv_device_fault" in e for e in check_bindings(bad, protos))
    # CInt where the C side takes size_t
    bad = good.replace("c_hkv_verify :: Ptr HkvCtx -> Ptr HkvBatch -> CSize ->",
                       "c_hkv_verify :: Ptr HkvCtx -> Ptr HkvBatch -> CInt ->")
    assert bad != good
    assert any("hkv_verify (" in e and "argument 3" in e for e in check_bindings(bad, protos))
    # a pointer to the wrong struct, a wrong result and an unknown symbol
    bad = good.replace("Ptr HkvTxs -> Ptr InputJob -> CSize -> Int32 -> Ptr Word32 -> IO CInt",
                       "Ptr InputJob -> Ptr HkvTxs -> CSize -> Int32 -> Ptr Word32 -> IO CInt")
    assert bad != good and len(check_bindings(bad, protos)) == 2
    bad = good.replace("c_hkv_close :: Ptr HkvCtx -> IO ()", "c_hkv_close :: Ptr HkvCtx -> IO CInt")
    assert any("result" in e for e in check_bindings(bad, protos))
    bad = good.replace('"hkv_batch_capacity"', '"hkv_batch_size"')
    assert any("not declared" in e for e in check_bindings(bad, protos))
