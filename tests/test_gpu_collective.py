"""The RCCL collective on hardware. `bench.py
--force-collective` at WORLD_SIZE 1 creates the nccl (= RCCL) process group
with device_id, as every N > 1 rank does, and keeps the step's device-side
all_gather_into_tensor of the verdict words (hkv/shard.py ShardedVerify.step)
on the stream libhkv enqueued the verify on. The gathered bitmap must equal
the labels, the rank's own words before the gather, and the bitmap of the same
configs[4] batch verified without any collective."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "HKV_BENCH_SPAWNED")}
    env["PYTHONUNBUFFERED"] = "1"
    return env


def _run(extra, tag):
    env = _env()
    if "--force-collective" in extra:
        env["NCCL_DEBUG"] = "VERSION"  # RCCL prints its version into the log
    # (output streamed to files under gpurun_out/ while the run goes)
    out = os.path.join(ROOT, "gpurun_out", f"collective_{tag}.log")
    err = os.path.join(ROOT, "gpurun_out", f"collective_{tag}.err")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as fo, open(err, "w") as fe:
        rc = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config4", "--steps", "3",
                             "--warmup", "1"] + extra, stdout=fo, stderr=fe, timeout=400, env=env, cwd=ROOT).returncode
    stdout, stderr = open(out).read(), open(err).read()
    assert rc == 0, stderr[-3000:]
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(900)
def test_rccl_all_gather_one_rank_equals_no_collective():
    rc = _run(["--gpus", "1", "--force-collective"], "rccl")
    assert rc["collective"] == "rccl" and rc["force_collective"] is True
    assert rc["ranks_seen"] == 1 and rc["n_gpus"] == 1
    assert rc["mismatches"] == 0 and rc["gather_vs_local_mismatches"] == 0
    assert rc["label_valid"] == rc["accepted"]
    assert "RCCL all-gather" in rc["config"]["workload"]
    plain = _run([], "none")
    assert plain["collective"] is None and plain["mismatches"] == 0
    assert plain["config"]["global_batch"] == rc["config"]["global_batch"] == 16777216
    assert plain["bitmap_sha256_128"] == rc["bitmap_sha256_128"]
    # the constant the N > 1 lines are checked against (bench.CONFIG4_BITMAP_SHA)
    assert rc["bitmap_equals_1gpu"] is True and plain["bitmap_equals_1gpu"] is True
