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
