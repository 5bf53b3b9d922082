"""Host build of the device safegcd inversion (hkv_safegcd.h: s^-1 mod n in
hkv_inv_kernel, den^-1 mod p in hkv_yverdict_kernel) against Python's
pow(x, -1, m): the same source the kernels compile, checked on edge and
random values."""
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


def build(tmp_path_factory, name, *defs):
    out = str(tmp_path_factory.mktemp("sgcd") / name)
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-Wno-unknown-pragmas", *defs, "-o", out,
                    os.path.join(ROOT, "tests", "safegcd_host.cpp")], check=True)
    return out


@pytest.fixture(scope="module")
def binary(tmp_path_factory):
    """The default build: the loop stops once g = 0 (HKV_SGCD_EARLY)."""
    return build(tmp_path_factory, "safegcd_host")


@pytest.fixture(scope="module")
def binary_full(tmp_path_factory):
    """All 25 iterations (HKV_SGCD_EARLY=0): what a lane that reached g = 0
    runs on the device while other lanes of its wave still iterate."""
    return build(tmp_path_factory, "safegcd_host_full", "-DHKV_SGCD_EARLY=0")


P = 2**256 - 2**32 - 977


def run(binary, xs, mod="n"):
    inp = "".join(f"{x:064x}\n" for x in xs)
    out = subprocess.run([binary, mod], input=inp, capture_output=True, text=True, check=True).stdout.split()
    return [int(h, 16) for h in out]


def test_safegcd_edge_scalars(binary):
    lam = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72
    xs = [1, 2, 3, N - 1, N - 2, (N - 1) // 2, (N + 1) // 2, 2**255, 2**128 - 1, 2**128, 2**128 + 1,
          2**32 - 1, 2**30, 2**30 - 1, 2**60 + 1, lam, N - lam, 0x10364141, 2**256 - 2**224 - 1 - N]
    xs = [x % N for x in xs if x % N]
    for x, r in zip(xs, run(binary, xs)):
        assert r == pow(x, -1, N), hex(x)


def test_safegcd_random(binary):
    rng = random.Random(0x5AFE)
    xs = [rng.randrange(1, N) for _ in range(20000)]
    xs += [rng.getrandbits(rng.randrange(1, 256)) or 1 for _ in range(5000)]   # short scalars
    xs += [N - (rng.getrandbits(rng.randrange(1, 128)) or 1) for _ in range(5000)]  # close to n
    for x, r in zip(xs, run(binary, xs)):
        assert r == pow(x, -1, N), hex(x)


def test_safegcd_zero_maps_to_zero(binary):
    assert run(binary, [0]) == [0]


def test_safegcd_mod_p(binary):
    rng = random.Random(0x50)
    xs = [1, 2, 3, P - 1, P - 2, (P - 1) // 2, 2**255, 2**32 + 977, 2**224, 0x3FFFFC2F, P - 2**32]
    xs += [rng.randrange(1, P) for _ in range(20000)]
    xs += [rng.getrandbits(rng.randrange(1, 256)) or 1 for _ in range(3000)]
    xs += [P - (rng.getrandbits(rng.randrange(1, 128)) or 1) for _ in range(3000)]
    for x, r in zip(xs, run(binary, xs, "p")):
        assert r == pow(x, -1, P), hex(x)


def test_safegcd_full_bound_equals_early_stop(binary, binary_full):
    """Divsteps after g = 0 are the identity on (f, d) mod the modulus, so the
    constant-time bound and the early stop give the same inverse."""
    rng = random.Random(0xE0)
    xs = [1, 2, 3, N - 1, 2**255, 2**128, 2**30] + [rng.randrange(1, N) for _ in range(5000)]
    xs += [rng.getrandbits(rng.randrange(1, 64)) or 1 for _ in range(2000)]
    assert run(binary, xs) == run(binary_full, xs) == [pow(x, -1, N) for x in xs]
    ps = [1, P - 1] + [rng.randrange(1, P) for _ in range(3000)]
    assert run(binary, ps, "p") == run(binary_full, ps, "p") == [pow(x, -1, P) for x in ps]


@pytest.fixture(scope="module")
def binary_flat(tmp_path_factory):
    """The device's branch-free divstep loop (HKV_SGCD_FLAT) built for the host."""
    return build(tmp_path_factory, "safegcd_host_flat", "-DHKV_SGCD_FLAT_HOST")


def test_safegcd_flat_loop_equals_branchy(binary, binary_flat):
    """The branch-free divsteps (the kernels' form) give the same inverses as
    the branchy form on edge and random scalars, mod n and mod p."""
    rng = random.Random(0x5F1A7)
    vals = [1, 2, 3, N - 1, N - 2, (N + 1) // 2, 1 << 128, (1 << 255) % N] + [rng.randrange(1, N) for _ in range(3000)]
    P = (1 << 256) - (1 << 32) - 977
    pv = [1, 2, P - 1, (1 << 200) + 7] + [rng.randrange(1, P) for _ in range(2000)]
    for mod, xs, m in (("n", vals, N), ("p", pv, P)):
        a, b = run(binary, xs, mod), run(binary_flat, xs, mod)
        assert a == b
        assert all(x * y % m == 1 for x, y in zip(xs, b))

