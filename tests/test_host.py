"""CPU tests of the host-side logic: record packing, bitmap unpacking, the
multi-GPU shard partition and the bench's verdict assembly."""
import numpy as np
import pytest

import secp256k1_oracle as o
from hkv import make_record, pack_records, unpack_bits
from hkv.records import bits_from_bools
from hkv.shard import shard_bounds


def test_record_layout_matches_oracle():
    msg = bytes(range(32))
    sig = bytes(range(64, 128))
    pk = bytes([2]) + bytes(range(100, 132))
    assert make_record(msg, sig, pk) == o.make_record(msg, sig, pk)
    arr = pack_records([(msg, sig, pk)] * 3)
    assert arr.shape == (3, 168) and arr[2, 96] == 33 and arr[2, 97] == 2


def test_record_validation():
    with pytest.raises(ValueError):
        make_record(b"x" * 31, b"y" * 64, b"")
    with pytest.raises(ValueError):
        make_record(b"x" * 32, b"y" * 63, b"")
    with pytest.raises(ValueError):
        make_record(b"x" * 32, b"y" * 64, b"z" * 66)


@pytest.mark.parametrize("n", [0, 1, 31, 32, 33, 64, 1000])
def test_bits_roundtrip(n):
    rng = np.random.default_rng(n)
    v = rng.random(n) < 0.5
    w = bits_from_bools(v)
    assert (unpack_bits(w, n) == v).all()


@pytest.mark.parametrize("n,world", [(0, 1), (1, 2), (100, 2), (1 << 20, 8), (16 * 2**20, 8), (1000, 3),
                                     (63, 4), (4000, 8)])
def test_shard_bounds_partition(n, world):
    b = [shard_bounds(n, r, world) for r in range(world)]
    assert b[0][0] == 0 and b[-1][1] == n
    for r in range(world - 1):
        assert b[r][1] == b[r + 1][0]
        assert b[r][0] % 64 == 0 or b[r][0] == b[r][1]  # 64-aligned non-empty starts
    assert all(lo <= hi for lo, hi in b)


def test_haskell_binding_layout_matches_ctypes_mirror():
    """haskell/Haskoin/Node/Verify{,/FFI}.hs (uncompiled here: no GHC) and the
    ctypes mirror (hkv/lib.py, hkv/records.py) describe the same bytes: the
    Storable offsets of HkvTxs / InputJob equal the ctypes field offsets, and
    pokeRecord's record offsets equal make_record's layout."""
    import ctypes
    import os
    import re
    from hkv.lib import HKV_RECORD_SIZE, HkvInputJob, HkvTxs
    from hkv.records import make_record
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ffi = open(os.path.join(root, "haskell", "Haskoin", "Node", "Verify", "FFI.hs")).read()
    ver = open(os.path.join(root, "haskell", "Haskoin", "Node", "Verify.hs")).read()

    def poke_offsets(instance):
        body = ffi[ffi.index(f"instance Storable {instance}"):]
        body = body[:body.index("\n\n")]
        size = int(re.search(r"sizeOf _ = (\d+)", body).group(1))
        return size, [int(x) for x in re.findall(r"pokeByteOff p (\d+)", body)]

    for inst, cstruct in (("HkvTxs", HkvTxs), ("InputJob", HkvInputJob)):
        size, offs = poke_offsets(inst)
        assert size == ctypes.sizeof(cstruct), inst
        assert offs == [getattr(cstruct, f[0]).offset for f in cstruct._fields_], inst
    assert f"hkvRecordSize = {HKV_RECORD_SIZE}" in ffi
    # pokeRecord: msg32 at 0, r||s at 32, pubkey length byte at 96, key at 97 (<= 65 bytes)
    assert "copyPrefix p 0 32 msg" in ver and "copyPrefix p 32 64 sig" in ver
    assert "pokeByteOff p 96" in ver and "copyPrefix p 97 65 pub" in ver
    rec = make_record(bytes(range(32)), bytes(range(32, 96)), b"\x02" + bytes(32))
    assert rec[:32] == bytes(range(32)) and rec[32:96] == bytes(range(32, 96))
    assert rec[96] == 33 and rec[97] == 2 and rec[130:] == bytes(HKV_RECORD_SIZE - 130)
