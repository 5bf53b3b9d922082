"""Benchmark: batch secp256k1 ECDSA verify on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Workload (BASELINE.json configs[1]): 1,048,576 synthetic valid secp256k1
(msg32, r, s, pubkey) records PER GPU (weak scaling; at N=8 this is the
configs[4] IBD shape, 8.4M signatures), generated on device by the keyless
construction (90% compressed / 10% uncompressed keys from a 65,536-key pool,
low-S) and resident in HBM before the timed region. One step = the full
verify of the rank's shard (prologue + ecmult + x-compare -> verdict bitmap)
plus, for N > 1, the RCCL all-gather of the verdict bitmap (the only
collective). value = all ranks' verifies / max-over-ranks time.

Also reported: verdict mismatches vs the construction labels (must be 0),
the ecmult kernel's roofline (integer limb products per verify from
hkv/opcount.py over the HIP-event-timed kernel duration, against the
measured v_mad_u64_u32 peak), and the CPU baseline: the C restatement
(oracle/, kind "port" — libsecp256k1 is not installed on the box) timed on the
host cores on a bounded sample.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "haskoin-node_amd"))

PER_GPU = 1 << 20
SEED = 0x484B5632
POOL = 65536
UNC_PERMILLE = 100


def cpu_baseline(records_host, threads: int):
    """Time the C oracle (checker port of the reference semantics) on the host."""
    import numpy as np
    so = os.path.join(ROOT, "oracle", "build", "libhkv_oracle.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, stdout=subprocess.DEVNULL)
    lib = ctypes.CDLL(so)
    lib.hkvo_verify_batch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.c_int]

    def run(n, t):
        out = np.zeros(n, dtype=np.uint8)
        t0 = time.perf_counter()
        lib.hkvo_verify_batch(ctypes.c_void_p(records_host.ctypes.data), n, 0, ctypes.c_void_p(out.ctypes.data), t)
        dt = time.perf_counter() - t0
        return n / dt, int(out.sum())

    n1 = 2048
    st_rate, ok1 = run(n1, 1)
    nm = min(len(records_host) // 168, 8192 * threads)
    mt_rate, okm = run(nm, threads)
    return {"value": round(mt_rate, 1), "unit": "verifies/s", "cores": threads, "kind": "port",
            "sample": f"{nm} of the timed config-2 records, HKV_LIBSECP semantics, {threads} pthreads "
                      f"(oracle/hkv_oracle.c; libsecp256k1 absent on the box)",
            "single_thread_value": round(st_rate, 1), "sample_accepts": okm, "sample_n": nm}


def block_mix(v, torch, sptr, steps: int) -> dict:
    """BASELINE configs[2]: a 2,000-tx P2PKH + P2WPKH block verified end to
    end on device (tx index, legacy / BIP143 sighash, DER + HASH160 template
    checks, ECDSA) from HBM-resident tx bytes; plus the same pipeline on a
    32-block batch (64,000 txs) for its throughput."""
    from hkv import blockgen
    out = {}
    # a dedicated stream: torch's default stream is the null stream (pointer 0),
    # which libhkv would replace by its own stream and the events would miss
    bstream = torch.cuda.Stream()
    sptr = bstream.cuda_stream
    for label, n_tx in (("block", 2000), ("batch32", 64000)):
        txs, inputs = blockgen.make_block(v, torch, n_tx=n_tx, seed=blockgen.SEED + n_tx)
        db = blockgen.DeviceBlock(torch, txs, inputs)

        def run():
            v.verify_std_inputs_device(0, db.txs, db.d_jobs.data_ptr(), db.n, -1, db.records.data_ptr(),
                                       db.bits.data_ptr(), sptr)

        def extract():
            v.std_inputs_device(0, db.txs, db.d_jobs.data_ptr(), db.n, -1, db.records.data_ptr(), sptr)

        run()
        torch.cuda.synchronize()
        words = db.bits.cpu().numpy().view("uint32")
        import numpy as np
        accepted = int(np.unpackbits(words.view(np.uint8), bitorder="little")[:db.n].sum())
        res = {"txs": n_tx, "inputs": db.n, "tx_bytes": int(db.d_bytes.numel()), "mismatches": db.n - accepted}
        for name, fn in (("total", run), ("extract_sighash", extract)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            k = max(3, steps // (1 if label == "block" else 4))
            e0.record(bstream)
            for _ in range(k):
                fn()
            e1.record(bstream)
            torch.cuda.synchronize()
            res[f"{name}_us"] = round(e0.elapsed_time(e1) * 1e3 / k, 1)
        res["inputs_per_s"] = round(db.n / (res["total_us"] * 1e-6), 1)
        out[label] = res
    out["workload"] = ("BASELINE configs[2]: 60% P2WPKH (BIP143) / 40% P2PKH (legacy) inputs, 1-3 inputs and 2 "
                       "outputs per tx, SIGHASH_ALL; verifyStdInput semantics, tx bytes resident in HBM")
    return out


def host_path(v, recs, n: int, steps: int) -> dict:
    """The drop-in boundary as the Haskell binding uses it: records in the
    pinned host batch (hkv_batch_alloc), hkv_verify = H2D (pipelined with the
    verify in grid-sized chunks) + kernels + D2H of the verdict words. This is
    the PCIe-inclusive rate; `value` stays the HBM-resident one."""
    import numpy as np
    b = ctypes.c_void_p()
    rc = v.lib.hkv_batch_alloc(v.ctx, n, ctypes.byref(b))
    if rc != 0:
        return {"error": rc}
    try:
        host = recs[: n * 168].cpu().numpy()
        dst = v.lib.hkv_batch_records(b)
        ctypes.memmove(dst, host.ctypes.data, n * 168)
        words = np.zeros((n + 31) // 32, dtype=np.uint32)
        wp = words.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
        v.lib.hkv_verify(v.ctx, b, n, 0, wp)
        k = max(3, steps // 2)
        t0 = time.perf_counter()
        for _ in range(k):
            v.lib.hkv_verify(v.ctx, b, n, 0, wp)
        dt = (time.perf_counter() - t0) / k
        acc = int(np.unpackbits(words.view(np.uint8), bitorder="little")[:n].sum())
        return {"records": n, "ms": round(dt * 1e3, 3), "verifies_per_s": round(n / dt, 1), "mismatches": n - acc,
                "h2d_bytes": n * 168, "note": "pinned host batch -> hkv_verify (blocking), PCIe-inclusive"}
    finally:
        v.lib.hkv_batch_free(b)


def header_batches(v, torch, steps: int) -> dict:
    """importHeaders' per-header work (headerHash +
    isValidPOW + linkage) for a 2,000-header peer message (a chained bchRegTest
    batch, hashed on the host with hashlib to build the links) and for 1M
    HBM-resident random headers (throughput)."""
    import hashlib
    import numpy as np
    from hkv import headers as hh
    limit = (1 << 255) - 1  # bchRegTest powLimit
    rng = np.random.default_rng(0x48445231)
    out = {}
    stream = torch.cuda.Stream()
    sp = stream.cuda_stream
    for label, n in (("message2000", 2000), ("batch1m", 1 << 20)):
        raw = rng.integers(0, 256, size=(n, 80), dtype=np.uint8)
        raw[:, 72:76] = np.frombuffer((0x207FFFFF).to_bytes(4, "little"), dtype=np.uint8)
        if label == "message2000":
            for i in range(1, n):
                raw[i, 4:36] = np.frombuffer(hashlib.sha256(hashlib.sha256(raw[i - 1].tobytes()).digest()).digest(),
                                             dtype=np.uint8)
        d = torch.from_numpy(raw.reshape(-1)).cuda()
        lim = torch.from_numpy(np.frombuffer(limit.to_bytes(32, "little"), dtype=np.uint8).copy()).cuda()
        hashes = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
        status = torch.zeros(n, dtype=torch.uint8, device="cuda")

        def run():
            hh.check_headers_device(v, 0, d.data_ptr(), n, lim.data_ptr(), None, hashes.data_ptr(),
                                    status.data_ptr(), sp)
        run()
        torch.cuda.synchronize()
        st = status.cpu().numpy()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        k = max(5, steps)
        e0.record(stream)
        for _ in range(k):
            run()
        e1.record(stream)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / k
        res = {"headers": n, "us": round(us, 1), "headers_per_s": round(n / (us * 1e-6), 1),
               "pow_ok": int((st & hh.HKV_HDR_POW_OK).astype(bool).sum())}
        if label == "message2000":
            res["linked"] = int((st & hh.HKV_HDR_LINK_OK).astype(bool).sum())
        out[label] = res
    out["workload"] = ("SURVEY §8(f) rank 4: importHeaders (Chain.hs:500-520) headerHash + isValidPOW + prev "
                       "linkage, bchRegTest bits 0x207fffff, headers resident in HBM")
    return out


def adversarial_mix(v, torch, recs, n: int, sptr: int, steps: int) -> dict:
    """BASELINE configs[3]: the timed batch with 30% of its records mutated into
    the SURVEY §8(c) invalid classes (hkv/adversarial.py: labels fixed by
    construction), verified in both modes; mismatches must be 0."""
    import numpy as np
    from hkv import adversarial
    adv, lab_lib, lab_hask, _ = adversarial.mutate(recs.cpu().numpy(), seed=0x484B5634)
    d = torch.from_numpy(adv).to(recs.device)
    words = torch.zeros((n + 63) // 64 * 2, dtype=torch.int32, device=recs.device)
    stream = torch.cuda.current_stream()
    out = {"records": n, "invalid_frac": round(float(1 - lab_lib.mean()), 4)}
    for name, mode, lab in (("libsecp", 0, lab_lib), ("haskoin", 1, lab_hask)):
        v.verify_device(0, d.data_ptr(), n, mode, words.data_ptr(), sptr)
        torch.cuda.synchronize()
        got = adversarial.unpack_bits(words.cpu().numpy().view(np.uint32), n)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        k = max(3, steps // 2)
        e0.record(stream)
        for _ in range(k):
            v.verify_device(0, d.data_ptr(), n, mode, words.data_ptr(), sptr)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / k
        out[name] = {"mismatches": int((got != lab).sum()), "accepts": int(got.sum()),
                     "ms": round(ms, 4), "verifies_per_s": round(n / (ms * 1e-3), 1)}
    out["workload"] = ("BASELINE configs[3]: msg-bit / r=0 / s>=n / bad prefix / x>=p / high-S mutations of "
                       "the config-2 records, labels by construction")
    return out


def merkle_batches(v, torch, steps: int) -> dict:
    """Block merkle roots (buildMerkleRoot, NodeSpec.hs:185-193) on HBM-resident
    txids: one 2,000-tx block (latency) and 4,096 blocks of 2,000 txs
    (throughput). Work: n-1 inner nodes per n-tx block, 3 SHA-256 compressions
    per node."""
    import numpy as np
    from hkv import merkle as mk
    rng = np.random.default_rng(0x4D4B4C31)
    out = {}
    stream = torch.cuda.Stream()
    sp = stream.cuda_stream
    for label, nb, ntx in (("block2000", 1, 2000), ("batch4096", 4096, 2000)):
        offsets = (np.arange(nb + 1, dtype=np.int64) * ntx).astype(np.int32)
        nl = nb * ntx
        dl = torch.from_numpy(rng.integers(0, 256, size=nl * 32, dtype=np.uint8)).cuda()
        do = torch.from_numpy(offsets).cuda()
        sc = torch.zeros(nl * 32, dtype=torch.uint8, device="cuda")
        dr = torch.zeros(nb * 32, dtype=torch.uint8, device="cuda")
        dm = torch.zeros(nb, dtype=torch.uint8, device="cuda")

        def run():
            mk.merkle_roots_device(v, 0, dl.data_ptr(), do.data_ptr(), nb, sc.data_ptr(), dr.data_ptr(),
                                   dm.data_ptr(), sp)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        k = max(5, steps)
        e0.record(stream)
        for _ in range(k):
            run()
        e1.record(stream)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / k
        nodes = nb * (ntx - 1)
        out[label] = {"blocks": nb, "txs_per_block": ntx, "us": round(us, 1),
                      "blocks_per_s": round(nb / (us * 1e-6), 1), "nodes_per_s": round(nodes / (us * 1e-6), 1),
                      "mutated": int(dm.sum().item())}
    out["workload"] = ("buildMerkleRoot per block (NodeSpec.hs:185-193 / haskoin-core Merkle [dep]), random "
                       "txids resident in HBM, one workgroup per block")
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--per-gpu", type=int, default=PER_GPU)
    ap.add_argument("--mode", type=int, default=0, help="0 = HKV_LIBSECP, 1 = HKV_HASKOIN")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-block-mix", action="store_true")
    ap.add_argument("--no-adversarial", action="store_true")
    ap.add_argument("--no-headers", action="store_true")
    ap.add_argument("--no-merkle", action="store_true")
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "latest_pmc_traffic.json"))
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)

    import hkv
    from hkv import opcount
    from hkv.shard import assemble_bitmap, shard_bounds

    n_total = args.per_gpu * world
    lo, hi = shard_bounds(n_total, rank, world)
    n = hi - lo
    v = hkv.Verifier(hkv.VerifierConfig(device_ids=[local]))
    # a real (non-null) stream made current: libhkv enqueues on it and the RCCL
    # all-gather, which waits on torch's current stream, is ordered after the
    # verify (the null stream would not order against libhkv's own stream)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    recs = torch.empty(n * 168, dtype=torch.uint8, device="cuda")
    # each rank generates exactly its slice of the global synthetic batch
    v.gen_records_device(0, SEED + lo, n, POOL, UNC_PERMILLE, recs.data_ptr(), sptr)
    words_per_rank = (args.per_gpu + 63) // 64 * 2 + 2
    bits = torch.zeros(words_per_rank, dtype=torch.int32, device="cuda")
    gathered = torch.zeros(words_per_rank * world, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()

    def step():
        v.verify_device(0, recs.data_ptr(), n, args.mode, bits.data_ptr(), sptr)
        if world > 1:
            dist.all_gather_into_tensor(gathered, bits)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    v.lib.hkv_profile_enable(v.ctx, 1)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    pm, em, nl = ctypes.c_double(), ctypes.c_double(), ctypes.c_uint64()
    v.lib.hkv_profile_read(v.ctx, 0, ctypes.byref(pm), ctypes.byref(em), ctypes.byref(nl))
    v.lib.hkv_profile_enable(v.ctx, 0)

    t = torch.tensor([dt, em.value / max(1, nl.value), pm.value / max(1, nl.value)], dtype=torch.float64,
                     device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt_max, ecm_ms, pro_ms = t.tolist()

    # correctness on the timed batch: every constructed signature is valid
    words = (gathered if world > 1 else bits).cpu().numpy().view(np.uint32)
    if world > 1:
        full = assemble_bitmap(n_total, world, words, words_per_rank)
    else:
        full = words[: (n + 31) // 32]
    accepted = int(np.unpackbits(full.view(np.uint8), bitorder="little")[:n_total].sum())
    mismatches = n_total - accepted

    if rank == 0:
        value = n_total * args.steps / dt_max
        per_launch_products = opcount.ECMULT_PRODUCTS_PER_VERIFY * n
        achieved = per_launch_products / (ecm_ms * 1e-3) / 1e12
        peak = opcount.PEAK_PRODUCTS_PER_S / 1e12
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                tj = json.load(open(args.traffic_json))
                if tj.get("per_verify_records") == n:
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        mix = None
        if world == 1 and not args.no_block_mix:
            mix = block_mix(v, torch, sptr, args.steps)
        hp = None
        if world == 1 and not args.no_host_path:
            hp = host_path(v, recs, n, args.steps)
        hdr = None
        if world == 1 and not args.no_headers:
            hdr = header_batches(v, torch, args.steps)
        mkl = None
        if world == 1 and not args.no_merkle:
            mkl = merkle_batches(v, torch, args.steps)
        adv = None
        if world == 1 and not args.no_adversarial:
            adv = adversarial_mix(v, torch, recs, n, sptr, args.steps)
        cpu = None
        if not args.no_cpu_baseline:
            host = recs[: min(n, 8192 * 16) * 168].cpu().numpy()
            threads = min(16, os.cpu_count() or 1)
            cpu = cpu_baseline(host, threads)
        line = {
            "metric": "ECDSA verifies/sec (1/8 GPU) + verdict mismatches vs libsecp256k1",
            "value": round(value, 1),
            "unit": "verifies/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (256-bit integer limbs)",
            "data": "synthetic (keyless-constructed valid secp256k1 tuples, generated on device)",
            "config": {"workload": "BASELINE configs[1]: 1,048,576 valid (hash,r,s,pubkey) per GPU, "
                                   "90% compressed / 10% uncompressed keys, 65,536-key pool; N>1 shards by "
                                   "signature index + RCCL verdict-bitmap all-gather",
                       "global_batch": n_total, "per_gpu": n, "mode": "LIBSECP" if args.mode == 0 else "HASKOIN",
                       "parallelism": f"dp{world}"},
            "mismatches": mismatches,
            "kernel_ms": {"prologue": round(pro_ms, 4), "ecmult": round(ecm_ms, 4)},
            "roofline": {"bound": "valu_int", "achieved": round(achieved, 4), "peak": round(peak, 3),
                         "unit": "T limb-products/s (v_mad_u64_u32)", "frac": round(achieved / peak, 4),
                         "traffic": traffic,
                         "kernel": "hkv_ecmult_kernel",
                         "products_per_verify": opcount.ECMULT_PRODUCTS_PER_VERIFY},
            "cpu_baseline": cpu,
            "block_mix": mix,
            "adversarial": adv,
            "headers": hdr,
            "merkle": mkl,
            "host_path": hp,
        }
        print(json.dumps(line), flush=True)
    v.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
