"""CPU-only sanitizer build of the host path's shard planning, bitmap merge
and device failover (haskoin-node_amd/csrc/hkv_plan.h, the code hkv_api.cpp
verify_from_host runs): tests/host_plan.cpp drives it with mock devices that
fail at enqueue or at join on a random schedule, under AddressSanitizer and
UndefinedBehaviorSanitizer (any report aborts the run). Checked: shards cover
the batch contiguously with 64-aligned starts; after any failure schedule
that leaves a device healthy every record is verified exactly once and every
verdict bit lands in place (nothing written past the bitmap); a round never
puts two shards on one device; failed devices are reported once and never
used again; with no healthy device the call fails without partial output."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_plan_and_failover_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_plan")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-fno-omit-frame-pointer",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-o", exe,
                    os.path.join(ROOT, "tests", "host_plan.cpp")], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok "), r.stdout
    assert int(r.stdout.split()[1]) > 20000
