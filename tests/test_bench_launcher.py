"""bench.py's launcher contract, on the CPU:

- `python bench.py --gpus 2` without a launcher starts two rank processes
  itself; both join the gloo group, run the sharded step with the one
  all-gather, and rank 0 prints ONE line with n_gpus = ranks_seen = 2 and
  both ranks' devices (the `--mock-cpu` leg writes a fixed verdict pattern
  instead of calling hkv_verify_device, and the gathered bitmap is checked
  against it);
- under a launcher, --gpus must equal WORLD_SIZE;
- --gpus N with fewer than N visible GPUs exits non-zero at once (this
  container has none)."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "HKV_BENCH_SPAWNED")}
    env.update(kw)
    return env


@pytest.mark.parametrize("world,n", [(2, 4096 + 65), (3, 64 * 10 + 7)])
def test_spawn_path_runs_every_rank(world, n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(world), "--mock-cpu", "--steps", "2", "--warmup", "1",
                        "--config4-n", str(n)], capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["mock"] is True
    assert d["n_gpus"] == world and d["ranks_seen"] == world
    assert sorted(x["rank"] for x in d["rank_devices"]) == list(range(world))
    assert len({x["pid"] for x in d["rank_devices"]}) == world  # distinct processes
    assert d["mismatches"] == 0 and d["global_batch"] == n


def test_gpus_must_match_world_size():
    t0 = time.time()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--mock-cpu"], capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
    assert time.time() - t0 < 60


def test_more_gpus_than_visible_fails_fast():
    """No GPU here: --gpus 2 must stop in the parent before starting ranks."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("two GPUs visible")
    t0 = time.time()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1"], capture_output=True, text=True,
                       timeout=120, env=_env())
    assert r.returncode == 2
    assert "GPU(s) visible" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert time.time() - t0 < 60


def test_failing_rank_stops_the_launch():
    """A rank that exits non-zero makes the launcher exit non-zero (the other
    rank is killed by PID rather than left waiting in the rendezvous)."""
    t0 = time.time()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--mock-cpu", "--config4-n", "4096"],
                       capture_output=True, text=True, timeout=120, env=_env(HKV_MOCK_FAIL_RANK="1"))
    assert r.returncode == 3
    assert "stopping the others" in r.stderr
    assert time.time() - t0 < 90


def test_force_collective_keeps_the_gather_at_one_rank():
    """--force-collective at WORLD_SIZE 1 (no launcher): the one-rank group is
    created and the step's all-gather runs (gloo in the mock leg; the GPU leg
    creates the nccl group, tests/test_gpu_collective.py), and the gathered
    bitmap equals the rank's own words and the pattern."""
    n = 4096 + 97
    r = subprocess.run([sys.executable, BENCH, "--mock-cpu", "--force-collective", "--steps", "2", "--warmup", "1",
                        "--config4-n", str(n)], capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["collective"] == "gloo" and d["n_gpus"] == 1
    assert d["mismatches"] == 0 and d["gather_vs_local_mismatches"] == 0
    r = subprocess.run([sys.executable, BENCH, "--mock-cpu", "--steps", "1", "--warmup", "0",
                        "--config4-n", str(n)], capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])["collective"] is None
