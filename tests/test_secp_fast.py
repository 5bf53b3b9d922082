"""The libsecp256k1-class CPU stand-in (oracle/secp_fast.c, bench.py's
cpu_baseline fast leg) against the port (oracle/hkv_oracle.c) and the
fixtures (CPU only):

- every golden KAT class and the special pool (r + n branch, edge scalars,
  u1 = 0, msg >= n, sum = infinity, ladder collisions), both modes, equal to
  the manifest labels;
- every adversarial class of hkv.adversarial (configs[3]) and generated
  configs[4]-style batches (5-30% invalid), equal to the port and the labels;
- its s^-1 (variable-time safegcd) against pow(s, -1, n) on edge and random
  scalars, and its GLV split: k1 + k2 lambda == k (mod n), |k1|, |k2| < 2^129;
- it is the faster checker: >= 2x the port's single-thread rate here, under
  the parallel test load (3.4x on the GPU box's host, profiles/r04a_bench.log)."""
import ctypes
import json
import os
import random
import time

import numpy as np
import pytest

import secp256k1_oracle as o
from conftest import GOLDEN, ROOT, c_gen_batch, fast_batch, oracle_batch
from hkv import adversarial

@pytest.fixture(scope="module")
def fast(secpfast):
    lib = secpfast
    lib.hkvo_fast_sc_inverse.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    lib.hkvo_fast_glv_split.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p]
    return lib


@pytest.mark.parametrize("mode,key", [(0, "libsecp"), (1, "haskoin")])
def test_golden_kats_and_special_pool(fast, mode, key):
    man = json.load(open(os.path.join(GOLDEN, "kat_manifest.json")))
    data = open(os.path.join(GOLDEN, "kat_records.bin"), "rb").read()
    got = fast_batch(fast, data, mode)
    exp = np.array([r[key] for r in man["records"]])
    bad = [man["records"][i]["class"] for i in np.nonzero(got != exp)[0]]
    assert not bad, bad
    sp = json.load(open(os.path.join(GOLDEN, "special_pool.json")))
    data = open(os.path.join(GOLDEN, "special_pool.bin"), "rb").read()
    got = fast_batch(fast, data, mode)
    exp = np.array([r[key] for r in sp["records"]])
    bad = sorted({sp["records"][i]["class"] for i in np.nonzero(got != exp)[0]})
    assert not bad, bad


def test_every_adversarial_class(fast, coracle):
    rng = random.Random(11)
    recs = []
    for i in range(64):
        q = o.point_mul(rng.randrange(1, o.N), o.G)
        m, r, s = o.keyless_tuple(rng.randrange(1, o.N), rng.randrange(1, o.N), q)
        if s > o.N // 2:
            s = o.N - s
        recs.append(o.make_record(m, r.to_bytes(32, "big") + s.to_bytes(32, "big"), o.pubkey_serialize(q, i % 5 != 0)))
    base = np.frombuffer(b"".join(recs), dtype=np.uint8)
    adv, lib_lab, hask_lab, cls = adversarial.mutate(np.tile(base, 30), seed=17, invalid_frac=0.7, special_frac=0.2)
    for mode, lab in ((0, lib_lab), (1, hask_lab)):
        got = fast_batch(fast, adv, mode)
        assert (got == oracle_batch(coracle, adv.tobytes(), mode)).all()
        bad = sorted({adversarial.CLASSES[c] for c in cls[got != lab]})
        assert not bad, (mode, bad)


@pytest.mark.parametrize("seed,inv", [(0x484B5635, 50), (0x1234, 300)])
def test_generated_batches_equal_port(fast, coracle, seed, inv):
    recs, lab, _ = c_gen_batch(coracle, seed, 4096, 2000, 64, 100, inv)
    for mode in (0, 1):
        got = fast_batch(fast, recs, mode)
        assert (got == oracle_batch(coracle, recs.tobytes(), mode)).all()
        assert (got == lab).all()


def test_scalar_inverse(fast):
    rng = random.Random(5)
    vals = [1, 2, 3, o.N - 1, o.N - 2, o.N // 2, 2**128, 2**255 % o.N, (1 << 62) - 1, 1 << 62, 1 << 124]
    vals += [rng.randrange(1, o.N) for _ in range(3000)]
    out = ctypes.create_string_buffer(32)
    for v in vals:
        fast.hkvo_fast_sc_inverse(v.to_bytes(32, "big"), out)
        assert int.from_bytes(out.raw, "big") == pow(v, -1, o.N), hex(v)


def test_glv_split(fast):
    lam = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72
    rng = random.Random(6)
    vals = [0, 1, o.N - 1, lam, o.N - lam, (o.N - 1) // 2] + [rng.randrange(o.N) for _ in range(3000)]
    m1 = (ctypes.c_uint64 * 3)()
    m2 = (ctypes.c_uint64 * 3)()
    s1, s2 = ctypes.c_int(), ctypes.c_int()
    for k in vals:
        fast.hkvo_fast_glv_split(k.to_bytes(32, "big"), m1, ctypes.byref(s1), m2, ctypes.byref(s2))
        a = m1[0] | m1[1] << 64 | m1[2] << 128
        b = m2[0] | m2[1] << 64 | m2[2] << 128
        assert a < 2**129 and b < 2**129
        assert (s1.value * a + s2.value * b * lam - k) % o.N == 0


def test_faster_than_port(fast, coracle):
    """The point of the stand-in: of the reference library's class (GLV,
    w = 15 G tables, safegcd), well above the port's rate on one thread (best
    of three runs of each)."""
    recs, _, _ = c_gen_batch(coracle, 0x484B5632, 0, 1200, 64, 100, 0)

    def rate(fn):
        out = np.zeros(1200, dtype=np.uint8)
        best = 0.0
        for _ in range(3):
            t0 = time.perf_counter()
            fn(recs.ctypes.data_as(ctypes.c_void_p), 1200, 0, out.ctypes.data_as(ctypes.c_void_p), 1)
            best = max(best, 1200 / (time.perf_counter() - t0))
        assert out.all()
        return best

    assert rate(fast.hkvo_fast_verify_batch) >= 2 * rate(coracle.hkvo_verify_batch)


def test_cpu_baseline_reports_both_whole_host_extrapolations(coracle, monkeypatch):
    """bench.py's CPU leg on a small sample (short points): the SMT-core
    point (1 thread on one CPU, then 2 threads on it and a sibling; the
    sibling pair is forced to two CPUs of this container's mask, which has no
    SMT) feeds whole_host.smt_extrapolated_value, and north_star_ratio quotes
    the stricter SMT ratio first and decides target_met_whole_host by it."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    aff = sorted(os.sched_getaffinity(0))
    if len(aff) < 2:
        pytest.skip("needs two CPUs")
    monkeypatch.setattr(bench, "smt_pair", lambda: (aff[0], aff[1]))
    monkeypatch.setattr(bench, "physical_cores", lambda info: 128)
    recs, _, _ = c_gen_batch(coracle, 0x484B5632, 0, 200, 64, 100, 0)
    cpu = bench.cpu_baseline([("s", recs, 1, None)], [1, 2], min_s=0.05)
    wh = cpu["whole_host"]
    smt = wh["smt_core"]
    assert smt["cpus"] == [aff[0], aff[1]] and smt["core_rate_smt"] > 0 and smt["core_rate_1t"] > 0
    assert wh["smt_extrapolated_value"] == round(smt["core_rate_smt"] * 128, 1)
    assert "UPPER bound" in cpu["kind_note"]
    assert os.sched_getaffinity(0) == set(aff)  # restored
    r = bench.north_star_ratio(1e8, cpu)
    assert list(r)[0] == "whole_host_smt_extrapolated"
    assert r["whole_host_smt_extrapolated"] == round(1e8 / wh["smt_extrapolated_value"], 1)
    assert r["target_met_whole_host"] == (r["whole_host_smt_extrapolated"] >= 50.0)


def test_bench_checker_leg_counts_mismatches(coracle, secpfast):
    """bench.py's mismatches_vs_checker leg: every record of the slice through
    secp_fast, compared bit for bit with the slice of the gathered bitmap —
    0 on the construction labels of a configs[4]-style slice, and a flipped
    verdict is counted."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    recs, lab, _ = c_gen_batch(coracle, 0x484B5635, 777_000, 2000, 65536, 100, 50)
    r = bench.checker_leg(recs, lab, 0)
    assert r["checked"] == 2000 and r["mismatches"] == 0 and r["checker"] == "oracle/secp_fast.c"
    bad = lab.copy()
    bad[[3, 1999]] ^= True
    assert bench.checker_leg(recs, bad, 0)["mismatches"] == 2
