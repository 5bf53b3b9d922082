"""The N > 1 bench code on a GPU: `bench.py --gpus 2
--share-device` on a 1-GPU lease starts two real rank processes from a
HIP-free parent (visible_devices() counts the KFD topology's render nodes,
no torch import), both open device 0 through libhkv, generate their slices
of the configs[4] batch on the device (hkv_gen_batch_device), verify them
with hkv_verify_device inside hkv.shard.ShardedVerify, all-gather the
verdict words (over gloo through host memory: RCCL takes one rank per GPU)
and check the gathered bitmap against the construction labels."""
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


def test_visible_devices_without_hip():
    sys.path.insert(0, ROOT)
    import bench
    import torch
    assert bench.visible_devices() == torch.cuda.device_count() >= 1


@pytest.mark.timeout(600)
def test_spawn_two_gpu_ranks_share_device():
    n = 2 * 1048576
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-device",
                        "--config4-n", str(n), "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=540, env=_env(), cwd=ROOT)
    log = os.path.join(ROOT, "gpurun_out", "spawn2.log")
    os.makedirs(os.path.dirname(log), exist_ok=True)
    with open(log, "w") as f:
        f.write(r.stdout + "\n--- stderr ---\n" + r.stderr)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["share_device"] is True
    assert d["launcher"] == "bench.py spawn"
    assert sorted(x["rank"] for x in d["rank_devices"]) == [0, 1]
    assert len({x["pid"] for x in d["rank_devices"]}) == 2
    assert all(x["device"] == 0 for x in d["rank_devices"])
    assert d["mismatches"] == 0
    assert d["config"]["global_batch"] == n and "configs[4]" in d["config"]["workload"]
    assert d["scaling"] == "strong"
    assert d["label_valid"] == d["accepted"] and 0.9 * n < d["accepted"] < n
