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


def _config4_worker(rank, world, port, n, seed, q):
    """One rank of bench.py's configs[4] leg on CPU: generate ONLY this rank's
    slice [lo, hi) of the global batch (the C restatement of
    hkv_gen_batch_device, index0 = lo, 5% invalid, construction labels),
    verify it (the C oracle stands in for hkv_verify_device), the one
    all-gather, then every rank checks its slice of the assembled bitmap
    against its labels and the counts are summed (all_reduce)."""
    import ctypes
    import sys
    import torch
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "..", "haskoin-node_amd"))
    sys.path.insert(0, here)
    from conftest import c_gen_batch
    from hkv.records import bits_from_bools
    from hkv.shard import ShardedVerify
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = ctypes.CDLL(ORACLE_SO)
    lib.hkvo_verify_batch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    holder = {}

    def cpu_verify(lo, hi, bits):
        out = np.zeros(hi - lo, dtype=np.uint8)
        recs = holder["recs"]
        lib.hkvo_verify_batch(recs.ctypes.data, hi - lo, 0, out.ctypes.data, 2)
        w = bits_from_bools(out.astype(bool))
        bits.zero_()
        bits[: len(w)] = torch.from_numpy(w.view(np.int32))

    sv = ShardedVerify(torch, n, rank, world, cpu_verify, dist=dist, device="cpu")
    recs, lab, _ = c_gen_batch(lib, seed, sv.lo, sv.local_n, 64, 100, 50)
    holder["recs"] = recs
    sv.step()
    full = sv.bitmap()
    t = torch.tensor([sv.slice_mismatches(full, bits_from_bools(lab)), int(lab.sum())], dtype=torch.int64)
    dist.all_reduce(t)
    if rank == 0:
        q.put((full.tobytes(), t.tolist()))
    dist.destroy_process_group()


@pytest.mark.parametrize("n,world", [(1500, 2), (64 * 9 + 33, 3)])
def test_config4_shards_generate_the_global_batch(n, world, coracle):
    """bench.py's configs[4] contract under gloo: ranks that each generate
    only their own slice produce the one-process batch, so the all-gathered
    bitmap equals the single-process bitmap of the whole batch and its
    construction labels bit for bit (mismatches summed over ranks = 0)."""
    from conftest import c_gen_batch
    seed = 0x484B5635
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_config4_worker, args=(r, world, port, n, seed, q)) for r in range(world)]
    for p in procs:
        p.start()
    got_bytes, (mism, accepts) = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = np.frombuffer(got_bytes, dtype=np.uint32)
    recs, lab, _ = c_gen_batch(coracle, seed, 0, n, 64, 100, 50)
    out = np.zeros(n, dtype=np.uint8)
    import ctypes
    coracle.hkvo_verify_batch(recs.ctypes.data_as(ctypes.c_void_p), n, 0, out.ctypes.data_as(ctypes.c_void_p), 8)
    exp = np.packbits(out, bitorder="little")
    exp = np.frombuffer(exp.tobytes() + b"\0" * ((-len(exp)) % 4), dtype=np.uint32)
    assert (got == exp).all()
    assert (out.astype(bool) == lab).all()
    assert mism == 0 and accepts == int(lab.sum()) and accepts < n


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
