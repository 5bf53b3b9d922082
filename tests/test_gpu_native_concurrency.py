"""Overlapping callers on one context from native C++ threads, with the C ABI
runtime (hkv_api.cpp: locks, per-device scratch order, streams) built plain,
under AddressSanitizer + UBSan and under ThreadSanitizer (host code only:
`-Xarch_host -fsanitize=...`, haskoin-node_amd/csrc/Makefile `sanitize`).
tools/native_concurrency.cpp: 6 threads mixing the host and device forms of
three blocks (configs[0], configs[2], a 600-input multisig block) and the
record entry points, every call's verdicts equal to a single-caller
reference, no fault status (the lock and stream logic had no
sanitizer build). The ROCm runtime is not instrumented; its internal races
are suppressed (tools/tsan.supp), libhkv's are not."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


@pytest.fixture(scope="module")
def blocks():
    dirs = []
    for name, which in (("nc_blk0", "config0"), ("nc_blk2", "config2"), ("nc_blkm", "multisig")):
        d = os.path.join(OUT, name)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "native_latency.py"), "dump", d, which],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        dirs.append(d)
    return dirs


@pytest.mark.timeout(900)
@pytest.mark.parametrize("variant,env,rounds", [
    ("", {}, 60),
    ("_asan", {"ASAN_OPTIONS": "detect_leaks=0:protect_shadow_gap=0:halt_on_error=1",
               "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}, 60),
    ("_tsan", {"TSAN_OPTIONS": "suppressions=" + os.path.join(ROOT, "tools", "tsan.supp") +
               ":halt_on_error=0:report_signal_unsafe=0:exitcode=66"}, 30),
])
def test_overlapping_native_callers(blocks, variant, env, rounds):
    tool = os.path.join(ROOT, "tools", "native_concurrency" + variant)
    if not os.access(tool, os.X_OK):
        pytest.fail(f"{tool} not built (make -C haskoin-node_amd/csrc sanitize)")
    r = subprocess.run([tool] + blocks + ["6", str(rounds)], capture_output=True, text=True, timeout=800,
                       env=dict(os.environ, **env))
    with open(os.path.join(OUT, f"native_concurrency{variant}.log"), "w") as f:
        f.write(r.stdout + "\n--- stderr ---\n" + r.stderr)
    # a sanitizer runtime that cannot lay out its shadow memory on this host's
    # address-space layout (e.g. TSan under high mmap randomisation) never
    # reaches libhkv: the host, not the code under test
    for fatal in ("ThreadSanitizer: unexpected memory mapping", "Shadow memory range interleaves"):
        if fatal in r.stderr and not r.stdout.strip():
            pytest.skip(f"{variant[1:]} runtime cannot start on this host: {fatal}")
    assert r.returncode == 0, r.stderr[-4000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
    assert "WARNING: ThreadSanitizer" not in r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["calls"] == 6 * rounds and d["mismatches"] == 0 and d["errors"] == 0 and d["faults"] == 0
    assert d["block_inputs"] == [4000, 3600, 600] and d["block_accepts"][:2] == [4000, 3600]
    assert 0 < d["block_accepts"][2] < 600
