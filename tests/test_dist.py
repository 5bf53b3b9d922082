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
    """One rank of the bench's multi-GPU step (hkv.shard.ShardedVerify: shard
    verify + the one all-gather + bitmap assembly), with the C oracle as the
    CPU stand-in for hkv_verify_device."""
    import ctypes
    import sys
    import torch
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "..", "haskoin-node_amd"))
    from hkv.records import bits_from_bools
    from hkv.shard import ShardedVerify
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data = open(os.path.join(GOLDEN, "kat_records.bin"), "rb").read()
    m = len(data) // 168
    recs = b"".join(data[(i % m) * 168:(i % m + 1) * 168] for i in range(n))
    lib = ctypes.CDLL(ORACLE_SO)

    def cpu_verify(lo, hi, bits):
        out = np.zeros(hi - lo, dtype=np.uint8)
        buf = np.frombuffer(recs[lo * 168:hi * 168], dtype=np.uint8)
        lib.hkvo_verify_batch(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(hi - lo), 1,
                              ctypes.c_void_p(out.ctypes.data), 2)
        w = bits_from_bools(out.astype(bool))
        bits.zero_()
        bits[: len(w)] = torch.from_numpy(w.view(np.int32))

    sv = ShardedVerify(torch, n, rank, world, cpu_verify, dist=dist, device="cpu")
    sv.step()
    full = sv.bitmap()
    if rank == 0:
        q.put(full.tobytes())
    dist.destroy_process_group()


@pytest.mark.parametrize("n,world", [(1000, 2), (64 * 7 + 5, 2), (3 * 64 + 1, 3)])
def test_two_rank_bitmap_equals_single(n, world, coracle):
    import ctypes
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
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
