"""World-size-2 gloo test (CPU) of the multi-GPU data path: index sharding +
one all-gather of the verdict bitmaps reproduces the single-process bitmap
bit for bit. The per-rank verifier here is the C oracle (checker); on the
GPU box each rank runs hkv_verify_device on its shard (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, ORACLE_SO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    import ctypes
    import sys
    import torch
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "..", "haskoin-node_amd"))
    from hkv.records import bits_from_bools
    from hkv.shard import assemble_bitmap, shard_bounds
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data = open(os.path.join(GOLDEN, "kat_records.bin"), "rb").read()
    m = len(data) // 168
    recs = b"".join(data[(i % m) * 168:(i % m + 1) * 168] for i in range(n))
    lo, hi = shard_bounds(n, rank, world)
    lib = ctypes.CDLL(ORACLE_SO)
    out = np.zeros(hi - lo, dtype=np.uint8)
    buf = np.frombuffer(recs[lo * 168:hi * 168], dtype=np.uint8)
    lib.hkvo_verify_batch(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(hi - lo), 1,
                          ctypes.c_void_p(out.ctypes.data), 2)
    wpr = (-(-n // world) + 63) // 64 * 2 + 2
    mine = np.zeros(wpr, dtype=np.uint32)
    w = bits_from_bools(out.astype(bool))
    mine[: len(w)] = w
    t = torch.from_numpy(mine.view(np.int32))
    gathered = torch.zeros(wpr * world, dtype=torch.int32)
    dist.all_gather_into_tensor(gathered, t)
    full = assemble_bitmap(n, world, gathered.numpy().view(np.uint32), wpr)
    if rank == 0:
        q.put(full.tobytes())
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [1000, 64 * 7 + 5])
def test_two_rank_bitmap_equals_single(n, coracle):
    import ctypes
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = np.frombuffer(q.get(timeout=120), dtype=np.uint32)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    data = open(os.path.join(GOLDEN, "kat_records.bin"), "rb").read()
    m = len(data) // 168
    recs = b"".join(data[(i % m) * 168:(i % m + 1) * 168] for i in range(n))
    out = np.zeros(n, dtype=np.uint8)
    buf = np.frombuffer(recs, dtype=np.uint8)
    coracle.hkvo_verify_batch(buf.ctypes.data_as(ctypes.c_void_p), n, 1, out.ctypes.data_as(ctypes.c_void_p), 4)
    exp = np.packbits(out, bitorder="little")
    exp = np.frombuffer(exp.tobytes() + b"\0" * ((-len(exp)) % 4), dtype=np.uint32)
    assert (got == exp).all()
