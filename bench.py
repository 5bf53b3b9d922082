"""Benchmark: batch secp256k1 ECDSA verify on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Without a launcher (WORLD_SIZE unset), --gpus N > 1 starts N rank processes
itself (fresh interpreters with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*; the
parent makes no GPU call) and exits non-zero at once when fewer than N GPUs
are visible. Under torchrun --gpus must equal WORLD_SIZE. The line carries
`ranks_seen` (dist.get_world_size()) and every rank's device.

Workloads (records generated on device by the keyless construction, 90%
compressed / 10% uncompressed keys from a 65,536-key pool, low-S, resident in
HBM before the timed region):
  N = 1 (the headline): BASELINE configs[1], 1,048,576 valid records
      (seed 0x484B5632); scaling "weak".
  N > 1 (torchrun), or --config4: BASELINE configs[4], ONE global batch of
      16,777,216 records (seed 0x484B5635, 5% mutated into rejecting
      classes), sharded by signature index (hkv/shard.py: contiguous,
      64-aligned; 2,097,152 per GPU at N = 8). Each rank generates only its
      slice, records [lo, hi) of that one batch (hkv_gen_batch_device: record
      k depends on (seed, k) only), with construction labels; scaling
      "strong" (the total is fixed).
One step = the verify of the rank's shard (prologue + ecmult + verdict ->
bitmap) plus, for N > 1, the RCCL all-gather of the verdict bitmap (the only
collective; hkv/shard.py ShardedVerify; --force-collective keeps it at N = 1
through a one-rank RCCL group, a test of the device collective on a 1-GPU
lease: the line then reads collective "rccl"). value = all ranks' verifies /
max-over-ranks time. After the timed steps every rank checks its slice of
the gathered bitmap against its labels and the counts are summed
(`mismatches`: every bit of the global bitmap against its record's label).

Also reported (rank 0, N = 1): the ecmult stage's roofline (the REFERENCE
algorithm's limb products per verify, hkv/opcount.py P_ALG_ECMULT, over the
HIP-event-timed ecmult + finish launches, against the v_mad_u64_u32 peak at 2.4 GHz and at the
measured mad rate and clock); configs[0] (the 2,000-tx P2PKH block), [2]
(block mix) and [3] (adversarial 1M, every class of hkv/adversarial.py); and
the CPU baseline leg: oracle/secp_fast.c, a restatement of libsecp256k1's
verify algorithm (GLV, w = 15 G tables, safegcd — the reference library's
class; libsecp256k1 is not installed on the box), timed in steady state (every
point >= 1 s of wall time, CPU seconds recorded) over a thread sweep (1, 16,
64, 128 and the affinity count) under the job's cgroup CPU quota, beside the
plain C restatement (oracle/hkv_oracle.c) and OpenSSL's ECDSA_do_verify; the
whole-host rate is extrapolated from the per-core rate and the host's
physical cores, and the north_star ratio is reported against both.
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
# BASELINE configs[4] / SURVEY §8(d) config 5: the IBD-style batch
CONFIG4_N = 1 << 24
CONFIG4_SEED = 0x484B5635
CONFIG4_INVALID_PERMILLE = 50
# SHA-256 (first 128 bits) of configs[4]'s global verdict bitmap (16,777,216
# records, the default seed / pool / invalid share, LIBSECP mode) as one GPU
# computes it, with and without the RCCL all-gather (profiles/r06a/, r06f/):
# SURVEY §8(e)'s check that the N-GPU bitmap is bit-identical to the 1-GPU one
CONFIG4_BITMAP_SHA = "3d2b3fc0ad2eacaae04c9f12bc5c16e0"


def cgroup_cpu_quota() -> dict:
    """This job's CPU quota as the kernel enforces it: cgroup v2 cpu.max
    ("max" or "<quota_us> <period_us>") or v1 cfs_quota_us / cfs_period_us."""
    out = {}
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us",
                 "/sys/fs/cgroup/cpu,cpuacct/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                out[path] = f.read().strip()
        except OSError:
            continue
    raw = out.get("/sys/fs/cgroup/cpu.max")
    if raw:
        q, _, per = raw.partition(" ")
        out["quota_cpus"] = None if q == "max" else round(int(q) / int(per or 100000), 2)
    else:
        q = out.get("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") or out.get("/sys/fs/cgroup/cpu,cpuacct/cpu.cfs_quota_us")
        if q is not None:
            out["quota_cpus"] = None if int(q) < 0 else round(int(q) / 100000, 2)
    return out


def host_info() -> dict:
    """lscpu model / topology of the box's host and this job's CPU share
    (affinity mask and cgroup quota)."""
    import subprocess
    info = {"os_cpu_count": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        pass
    info["cgroup"] = cgroup_cpu_quota()
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "CPU max MHz"):
                info[k.strip()] = v.strip()
    except Exception:  # pragma: no cover
        pass
    return info


def thread_sweep() -> list:
    """Thread counts of the all-core sweep: 1, 16, 64, 128 and every CPU the
    affinity mask allows (at most 256, the checkers' pthread cap)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        aff = os.cpu_count() or 1
    return sorted({t for t in (1, 16, 64, 128, aff) if t <= max(1, min(aff, 256))} | {min(aff, 256)})


def physical_cores(info: dict):
    """Physical cores of the whole host (lscpu sockets x cores per socket)."""
    try:
        return int(info["Socket(s)"]) * int(info["Core(s) per socket"])
    except (KeyError, ValueError):
        return None


def cpu_seconds() -> float:
    """CPU time (user + system) of this process, every thread included."""
    import resource
    ru = resource.getrusage(resource.RUSAGE_SELF)
    return ru.ru_utime + ru.ru_stime


def steady_rate(fn, recs, mode: int, threads: int, min_s: float, per_thread: int = 2000) -> dict:
    """Records/s of fn(records, n, mode, out, threads) in steady state: calls
    on `per_thread` records per thread (the sample tiled) repeated until at
    least min_s of wall time has passed — >= 10 periods of the cgroup's CFS
    quota, so a burst at the start of a period cannot inflate the rate — with
    the process's CPU seconds recorded beside the wall clock (per-core rate =
    records / CPU-s)."""
    import numpy as np
    n0 = len(recs) // 168
    m = max(n0, per_thread * threads)
    reps = -(-m // n0)
    buf = np.ascontiguousarray(np.tile(recs, reps)[: m * 168] if reps > 1 else recs)
    out = np.zeros(m, dtype=np.uint8)
    done, calls = 0, 0
    c0, t0 = cpu_seconds(), time.perf_counter()
    while True:
        fn(ctypes.c_void_p(buf.ctypes.data), m, mode, ctypes.c_void_p(out.ctypes.data), threads)
        done += m
        calls += 1
        wall = time.perf_counter() - t0
        if wall >= min_s:
            break
    cpu = cpu_seconds() - c0
    return {"threads": threads, "records": done, "calls": calls, "wall_s": round(wall, 3), "cpu_s": round(cpu, 3),
            "rate": round(done / wall, 1), "per_cpu_s": round(done / cpu, 1) if cpu > 0 else None,
            "verdicts": out[:n0].astype(bool)}


def smt_pair() -> tuple:
    """Two CPUs of this job's affinity mask that are SMT siblings of one
    physical core (sysfs thread_siblings_list), or None."""
    try:
        aff = sorted(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        return None
    for c in reversed(aff):  # (from the top: CPU 0 takes most of the host's interrupts)
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                txt = f.read().strip()
        except OSError:
            continue
        sib = set()
        for part in txt.split(","):
            a, _, b = part.partition("-")
            sib.update(range(int(a), int(b or a) + 1))
        others = sorted(x for x in sib if x != c and x in aff)
        if others:
            return c, others[0]
    return None


def smt_core_rate(fn, recs, mode: int, min_s: float) -> dict:
    """One physical core, measured: fn at 1 thread pinned to one CPU, then at
    2 threads pinned to that CPU and its SMT sibling (threads inherit the
    caller's affinity), each >= min_s in steady state. core_rate_smt is what
    one physical core delivers with both hardware threads busy."""
    pair = smt_pair()
    if pair is None:
        return {"skipped": "no SMT sibling pair in this job's affinity mask"}
    old = os.sched_getaffinity(0)
    try:
        os.sched_setaffinity(0, {pair[0]})
        one = steady_rate(fn, recs, mode, 1, min_s)
        os.sched_setaffinity(0, set(pair))
        two = steady_rate(fn, recs, mode, 2, min_s)
    finally:
        os.sched_setaffinity(0, old)
    one.pop("verdicts")
    two.pop("verdicts")
    return {"cpus": list(pair), "one_thread": one, "two_threads_smt": two, "core_rate_1t": one["rate"],
            "core_rate_smt": two["rate"], "smt_gain": round(two["rate"] / one["rate"], 3)}


def checker_leg(recs_host, got_bits, mode: int) -> dict:
    """Every record of this rank's slice re-verified on the host by
    oracle/secp_fast.c (the libsecp256k1-class restatement: GLV + wNAF, 5 x
    52-bit field, safegcd — the CPU baseline's implementation) and compared
    with this rank's slice of the gathered bitmap: the metric's "verdict
    mismatches vs libsecp256k1", against a checker rather than the
    construction labels. Outside the timed region; the oracle is only the
    checker here. Threads: this process's CPU share over the node's ranks,
    at most 16."""
    import numpy as np
    so = os.path.join(ROOT, "oracle", "build", "libhkv_secpfast.so")
    if not os.path.exists(so):
        return {"checked": 0, "mismatches": None, "note": "oracle/build/libhkv_secpfast.so not built"}
    fast = ctypes.CDLL(so)
    fast.hkvo_fast_verify_batch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_int]
    try:
        cpus = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        cpus = os.cpu_count() or 1
    threads = max(1, min(16, cpus // max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))))
    n = len(recs_host) // 168
    out = np.zeros(n, dtype=np.uint8)
    t0 = time.perf_counter()
    fast.hkvo_fast_verify_batch(np.ascontiguousarray(recs_host).ctypes.data, n, mode, out.ctypes.data, threads)
    dt = time.perf_counter() - t0
    mism = int(np.count_nonzero(out.astype(bool) != got_bits[:n]))
    return {"checked": n, "mismatches": mism, "threads": threads, "seconds": round(dt, 2),
            "checker": "oracle/secp_fast.c"}


def cpu_baseline(samples, sweep, min_s: float = 1.0) -> dict:
    """The CPU leg (oracle/ is timed here and used as the checker here only).

    samples: [(name, records uint8 [n*168], mode, gpu verdicts bool[n] or None)].
    Every timed point is a steady-state measurement (steady_rate: >= min_s of
    wall time, CPU seconds recorded). The reported baseline is "secpfast" =
    oracle/secp_fast.c, a restatement (port) of libsecp256k1's verify
    algorithm (5x52 field, GLV + wNAF5 Strauss, w = 15 G tables,
    variable-time safegcd s^-1) — the reference library's class; the library
    itself is not installed on the box. It is timed on the first sample
    (configs[0]'s block) at every thread count of `sweep`; `value` is the best
    steady rate (bound by the job's cgroup CPU quota) and `cores` the thread
    count that reached it. Beside it: "port" = oracle/hkv_oracle.c (plain C
    restatement; no GLV, generic inversions) and "openssl" = OpenSSL 3
    ECDSA_do_verify behind oracle/openssl_check.c (the survey's labelled
    non-reference fallback), each at 1 thread and at the quota's CPU count.
    The other samples are timed with secpfast at 1 thread; every
    implementation's verdicts on every sample are compared with the GPU's.
    The whole-host rate is an extrapolation: the per-core rate (records per
    CPU-second) x the host's physical cores (lscpu)."""
    import numpy as np
    import subprocess
    ob = os.path.join(ROOT, "oracle", "build")
    sos = ("libhkv_oracle.so", "libhkv_openssl.so", "libhkv_secpfast.so")
    if not all(os.path.exists(os.path.join(ob, x)) for x in sos):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, stdout=subprocess.DEVNULL)
    argt = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    port = ctypes.CDLL(os.path.join(ob, "libhkv_oracle.so"))
    port.hkvo_verify_batch.argtypes = argt
    ossl = ctypes.CDLL(os.path.join(ob, "libhkv_openssl.so"))
    ossl.hkvo_openssl_verify_batch.argtypes = argt
    fast = ctypes.CDLL(os.path.join(ob, "libhkv_secpfast.so"))
    fast.hkvo_fast_verify_batch.argtypes = argt
    impls = {"secpfast": fast.hkvo_fast_verify_batch, "port": port.hkvo_verify_batch,
             "openssl": ossl.hkvo_openssl_verify_batch}
    host = host_info()
    quota = host.get("cgroup", {}).get("quota_cpus")
    aff = host.get("affinity_cpus") or os.cpu_count() or 1
    q_threads = max(1, min(aff, int(quota) if quota else aff, 256))

    def point(fn, recs, mode, t):
        r = steady_rate(fn, recs, mode, t, min_s)
        v = r.pop("verdicts")
        return r, v

    res = {}
    best = None  # secpfast on the first sample: (rate, threads) of the sweep
    single = per_core = None
    quota_point = None  # secpfast at the quota's CPU count, >= 3 s: `value`
    for si, (name, recs, mode, gpu) in enumerate(samples):
        recs = np.ascontiguousarray(recs)
        n = len(recs) // 168
        row = {"records": n, "mode": "LIBSECP" if mode == 0 else "HASKOIN"}
        for iname, fn in impls.items():
            if si == 0:
                counts = sweep if iname == "secpfast" else sorted({1, q_threads})
            else:
                counts = [1] if iname == "secpfast" else []
            r = {}
            vm = None
            for t in counts:
                pt, v = point(fn, recs, mode, t)
                r[f"{t}_threads"] = pt
                vm = v if vm is None else vm
                if si == 0 and iname == "secpfast":
                    if best is None or pt["rate"] > best[0]:
                        best = (pt["rate"], t)
                    if t == 1:
                        single, per_core = pt["rate"], pt["per_cpu_s"]
            if vm is None:  # verdicts only (untimed)
                out = np.zeros(n, dtype=np.uint8)
                fn(ctypes.c_void_p(recs.ctypes.data), n, mode, ctypes.c_void_p(out.ctypes.data), q_threads)
                vm = out.astype(bool)
            r["accepts"] = int(vm.sum())
            if gpu is not None:
                r["mismatches_vs_gpu"] = int((vm != gpu).sum())
            row[iname] = r
        res[name] = row
    if not samples:
        return {"value": None, "unit": "verifies/s", "cores": None, "kind": "port", "impl": "secpfast"}
    # `value`: the steady rate at the quota's CPU count over >= 3 s (30 CFS
    # periods), the job's all-core share; the sweep's points run >= 1 s each
    # and are reported beside it (best_of_sweep)
    quota_point = steady_rate(impls["secpfast"], np.ascontiguousarray(samples[0][1]), samples[0][2], q_threads,
                              max(3.0, 3 * min_s))
    quota_point.pop("verdicts")
    quota_point["effective_cpus"] = round(quota_point["cpu_s"] / quota_point["wall_s"], 2)
    rate, cores = quota_point["rate"], q_threads
    phys = physical_cores(host)
    smt = smt_core_rate(impls["secpfast"], np.ascontiguousarray(samples[0][1]), samples[0][2], max(2.0, 2 * min_s))
    smt_rate = smt.get("core_rate_smt")
    first = samples[0][0]
    return {"value": rate, "unit": "verifies/s", "cores": cores, "kind": "port", "impl": "secpfast",
            "value_point": quota_point,
            "best_of_sweep": {"rate": best[0], "threads": best[1]},
            "kind_note": "a port of the reference library's algorithm: oracle/secp_fast.c restates libsecp256k1's "
                         "verify (5x52 field, GLV + wNAF5, w=15 G tables, safegcd, the pubkey parse / sqrt); "
                         "libsecp256k1 itself is not installed on the box and not in /root/reference. Its speed "
                         "relative to libsecp256k1 (x86-64 asm field, tuned tables) is unmeasured, so every GPU/CPU "
                         "ratio against it is an UPPER bound on the ratio against the real library",
            "sample": f"BASELINE configs[0]: the 4,000 inputs of the 2,000-tx P2PKH block (records extracted on "
                      f"device, HKV_HASKOIN = verifyHashSig), tiled to 2,000 records per thread per call; value = "
                      f"the steady rate at {cores} threads (this job's cgroup CPU quota, {quota} CPUs) over >= "
                      f"{max(3.0, 3 * min_s):g} s of wall time; the thread sweep {list(sweep)} (>= {min_s:g} s per "
                      f"point) is reported beside it",
            "single_thread_value": single,
            "per_core_value": per_core,
            "per_core_note": "records per CPU-second (getrusage) of the 1-thread point",
            "quota_cpus": quota,
            "quota_bound_value": rate,
            "quota_check": {"max_point": max(best[0], rate),
                            "bound": round(quota * single * 1.1, 1) if quota and single else None,
                            "ok": bool(max(best[0], rate) <= quota * single * 1.1) if quota and single else None,
                            "note": "no point may exceed quota x single-thread rate x 1.1 (steady state)"},
            "whole_host": {"physical_cores": phys,
                           "smt_extrapolated_value": round(smt_rate * phys, 1) if smt_rate and phys else None,
                           "extrapolated_value": round(per_core * phys, 1) if per_core and phys else None,
                           "smt_core": smt,
                           "note": "smt_extrapolated_value = one physical core's measured rate with both SMT "
                                   "threads busy (smt_core: 2 threads pinned to sibling CPUs) x the host's physical "
                                   "cores (lscpu); extrapolated_value = the 1-thread per-CPU-second rate x the "
                                   "physical cores (ignores SMT). Both are extrapolations, not measurements (the "
                                   "job may use only its cgroup quota); the SMT one is the higher CPU rate"},
            "thread_sweep": list(sweep), "samples": res, "host": host}


def north_star_ratio(value: float, cpu: dict) -> dict:
    """north_star: ">= 50x the all-core host libsecp256k1 verify rate on one
    MI355X". The whole-host figure is the extrapolation (per-core rate x
    physical cores); the quota-bound figure is what this job measured."""
    wh = (cpu.get("whole_host") or {}).get("extrapolated_value")
    whs = (cpu.get("whole_host") or {}).get("smt_extrapolated_value")
    out = {"whole_host_smt_extrapolated": round(value / whs, 1) if whs else None,
           "whole_host_extrapolated": round(value / wh, 1) if wh else None,
           "quota_bound": round(value / cpu["value"], 1) if cpu.get("value") else None,
           "single_thread": round(value / cpu["single_thread_value"], 1) if cpu.get("single_thread_value") else None,
           "target": 50.0}
    low = out["whole_host_smt_extrapolated"] or out["whole_host_extrapolated"]
    out["target_met_whole_host"] = bool(low >= 50.0) if low is not None else None
    out["note"] = ("value (configs[1], HBM-resident) / the CPU rates. The north_star reading is against all host "
                   "cores, extrapolated: whole_host_smt_extrapolated (each physical core with both SMT threads, "
                   "measured on one core) is the lower, stricter ratio and decides target_met_whole_host; "
                   "whole_host_extrapolated ignores SMT. Both are upper bounds against libsecp256k1 itself "
                   "(cpu_baseline.kind_note); quota_bound is against this job's cgroup CPU share (measured)")
    return out


def _time_block(v, torch, db, bstream, k: int) -> dict:
    """Verify one HBM-resident tx batch end to end (tx index, sighash, DER /
    template / HASH160 checks, ECDSA) on bstream; HIP-event times."""
    import numpy as np
    sptr = bstream.cuda_stream

    def run():
        v.verify_std_inputs_device(0, db.txs, db.d_jobs.data_ptr(), db.n, -1, db.records.data_ptr(),
                                   db.bits.data_ptr(), sptr)

    def extract():
        v.std_inputs_device(0, db.txs, db.d_jobs.data_ptr(), db.n, -1, db.records.data_ptr(), sptr)

    run()
    torch.cuda.synchronize()
    words = db.bits.cpu().numpy().view("uint32")
    got = np.unpackbits(words.view(np.uint8), bitorder="little")[:db.n].astype(bool)
    res = {"txs": db.n_tx, "inputs": db.n, "tx_bytes": int(db.d_bytes.numel()),
           "accepted": int(got.sum()), "rejected": int(db.n - got.sum())}
    # k calls back to back between two events, three times after at least
    # 100 ms of untimed calls; the median. Without the warm-up the first loop after a
    # data set's first call ran slow and each later one faster (configs[0]
    # 268 / 262 / 255 us, the 64,000-tx batch 1,521 / 1,445 / 1,407 us,
    # profiles/r04r_bench_reps.log), where 20 calls in, every timing method
    # agrees (events around 3, 10 or 32 calls, the host clock around 32, one
    # call alone: 255-258 and 1,378-1,395 us, tools/block_timing.py,
    # profiles/r04r_block_timing.txt). The reps stay in the line.
    for name, fn in (("total", run), ("extract_sighash", extract)):
        # warm-up: calls for at least 100 ms of wall time (with 20 calls the
        # three loops still ran 257 / 252 / 250 us on configs[0],
        # profiles/r04r_ix_bench.log: the clock ramps over tens of ms)
        t_w = time.perf_counter()
        while True:
            for _ in range(max(k, 10)):
                fn()
            torch.cuda.synchronize()
            if time.perf_counter() - t_w > 0.1:
                break
        reps = []
        for _ in range(3):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(bstream)
            for _ in range(k):
                fn()
            e1.record(bstream)
            torch.cuda.synchronize()
            reps.append(e0.elapsed_time(e1) * 1e3 / k)
        res[f"{name}_us"] = round(sorted(reps)[1], 1)
        res[f"{name}_us_reps"] = [round(x, 1) for x in reps]
    res["inputs_per_s"] = round(db.n / (res["total_us"] * 1e-6), 1)
    # one block at a time (the stream idle before each call): its latency
    lat = []
    for _ in range(max(3, k // 2)):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(bstream)
        run()
        e1.record(bstream)
        torch.cuda.synchronize()
        lat.append(e0.elapsed_time(e1) * 1e3)
    res["latency_us"] = round(sorted(lat)[len(lat) // 2], 1)
    # 32 blocks enqueued back to back (the device entry point only enqueues:
    # the host's clock runs from the first enqueue to the last verdict)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(32):
        run()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t32 = time.perf_counter() - t0
    res["back_to_back32"] = {"blocks_per_s": round(32 / t32, 1), "us_per_block": round(t32 / 32 * 1e6, 1),
                             "enqueue_us_per_block": round(t_enq / 32 * 1e6, 1),
                             "note": "32 calls of hkv_verify_std_inputs_device on one stream, no host sync between "
                                     "them; host wall clock from the first enqueue to the last verdict"}
    # (a block: one workgroup of the block kernel per 16 inputs). Other batch
    # sizes run other kernels, which leave no fresh stamps: null
    n_pad = (db.n + 255) // 256 * 256
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    res["split_phases_us"] = split_phases(v, torch, run, n_pad // 16) if n_pad <= 16 * n_cu else None
    return res, got


# phase slots of the block kernel (hkv_kernels.hip 2d): wave 0 (low windows),
# wave 1 (2^(4 K1) Q' / 2^(4 K2) Q' and the high windows), wave 2 (signature),
# wave 3 (key sqrt, then the middle windows)
PHASES = ("start", "lo_table", "digits", "lo_chain", "a_y0", "verdict", "sig_parse", "u1G", "key_sqrt",
          "hi_table", "hi_chain", "mid_chain")


def split_phases(v, torch, run, n_groups: int = 0) -> dict:
    """Phase boundaries of workgroup 0 of the small-batch kernel in one extra
    profiled call (hkv_profile_phases: constant-rate clock stamps,
    microseconds after the kernel's start)."""
    v.lib.hkv_profile_enable(v.ctx, 1)
    run()
    torch.cuda.synchronize()
    stamps = (ctypes.c_uint64 * len(PHASES))()
    tick = ctypes.c_double()
    v.lib.hkv_profile_phases(v.ctx, 0, stamps, len(PHASES), ctypes.byref(tick))
    out = {name: round((int(stamps[k]) - int(stamps[0])) * tick.value * 1e-3, 1) for k, name in enumerate(PHASES)}
    # every stamp of this call lies after its start and within the call: a
    # stamp outside that was not written by it
    bad = [name for name in PHASES if not 0.0 <= out[name] < 1e5]
    if bad:
        v.lib.hkv_profile_enable(v.ctx, 0)
        return {"error": f"stale or missing phase stamps: {bad}"}
    # every workgroup's (start, end) stamps (the block kernel only): how far
    # the launch's span reaches beyond workgroup 0's phase stamps
    if n_groups and hasattr(v.lib, "hkv_profile_group_stamps"):
        g = (ctypes.c_uint64 * (2 * n_groups))()
        v.lib.hkv_profile_group_stamps(v.ctx, 0, g, n_groups, ctypes.byref(tick))
        st_, en = [int(g[2 * k]) for k in range(n_groups)], [int(g[2 * k + 1]) for k in range(n_groups)]
        t0, us = min(st_), tick.value * 1e-3
        ends = sorted((e - t0) * us for e in en)
        out["groups"] = {"n": n_groups, "start_spread_us": round((max(st_) - t0) * us, 1),
                         "group0_start_us": round((st_[0] - t0) * us, 1),
                         "group0_end_us": round((en[0] - t0) * us, 1),
                         "end_min_us": round(ends[0], 1), "end_median_us": round(ends[len(ends) // 2], 1),
                         "end_max_us": round(ends[-1], 1)}
    v.lib.hkv_profile_enable(v.ctx, 0)
    return out


def block_mix(v, torch, steps: int, ibd_txs: int = 0) -> dict:
    """BASELINE configs[2]: a 2,000-tx P2PKH + P2WPKH block verified end to
    end on device from HBM-resident tx bytes; plus the same pipeline on a
    mempool-sized batch (9,000 txs, ~16,000 inputs: the pair kernel's range,
    4,097-32,768 inputs) and a 32-block batch (64,000 txs: the overlapped
    full-grid path) for their throughput; --std-ibd N adds one N-tx batch
    (e.g. 560,000 txs, ~1M inputs: an IBD-sized getBlocks list of blocks
    through the verifyStdInput path, sighash on device). Every generated
    input is valid; `rejected` must be 0 (the per-input records are checked
    against the oracle byte for byte in tests/test_gpu_sighash.py, not here)."""
    from hkv import blockgen
    out = {}
    # a dedicated stream: torch's default stream is the null stream (pointer 0)
    bstream = torch.cuda.Stream()
    sizes = [("block", 2000), ("pool16k", 9000), ("batch32", 64000)]
    if ibd_txs:
        sizes.append(("ibd", ibd_txs))
    for label, n_tx in sizes:
        txs, inputs = blockgen.make_block(v, torch, n_tx=n_tx, seed=blockgen.SEED + n_tx)
        db = blockgen.DeviceBlock(torch, txs, inputs)
        out[label], _ = _time_block(v, torch, db, bstream, max(5, steps // (1 if label == "block" else 4)))
    out["workload"] = ("BASELINE configs[2]: 60% P2WPKH (BIP143) / 40% P2PKH (legacy) inputs, 1-3 inputs and 2 "
                       "outputs per tx, SIGHASH_ALL; verifyStdInput semantics, tx bytes resident in HBM")
    return out


def config0_block(v, torch, steps: int):
    """BASELINE configs[0] on the GPU: the 2,000-tx x 2-input x 2-output P2PKH
    block (seed 0x484B5631, 4,096-key pool) verified end to end from
    HBM-resident tx bytes. Returns (result, device-extracted records, GPU
    verdicts, txs, inputs); the CPU leg times the same inputs on the host."""
    from hkv import blockgen
    txs, inputs = blockgen.make_p2pkh_block(v, torch)
    db = blockgen.DeviceBlock(torch, txs, inputs)
    bstream = torch.cuda.Stream()
    res, got = _time_block(v, torch, db, bstream, max(5, steps))
    recs = db.records[: db.n * 168].cpu().numpy().copy()
    res["workload"] = ("BASELINE configs[0]: 2,000 txs x 2 P2PKH inputs x 2 P2PKH outputs = 4,000 signatures, "
                       "seed 0x484B5631, compressed keys from a 4,096-key pool, SIGHASH_ALL, low S; "
                       "verifyStdInput semantics end to end on device")
    res["native_caller"] = native_caller(txs, inputs)
    return res, recs, got, txs, inputs


NATIVE = os.path.join(ROOT, "tools", "native_latency")


def native_caller(txs, inputs, calls: int = 20) -> dict:
    """The same block verified by a C++ caller through the C ABI only
    (tools/native_latency.cpp, a child process: no Python or ctypes in front
    of the call, as a Haskell node's FFI would call it): back to back, one
    call alone, one call alone after 5 ms of GPU idle (HIP events)."""
    import shutil
    import subprocess
    import tempfile
    import numpy as np
    from hkv.sighash import INPUT_JOB_DTYPE, TxBatch
    if not os.access(NATIVE, os.X_OK):
        return {"skipped": "tools/native_latency not built (make -C haskoin-node_amd/csrc)"}
    tb = TxBatch(txs)
    jobs = np.zeros(len(inputs), dtype=INPUT_JOB_DTYPE)
    for k, (t, i, spk, value) in enumerate(inputs):
        off, ln = tb.script(spk)
        jobs[k] = (t, i, off, ln, value)
    _, pool = tb.struct()
    d = tempfile.mkdtemp(prefix="hkv_blk_")
    try:
        for name, arr in (("txs", tb.bytes), ("offsets", tb.offsets), ("scripts", pool), ("jobs", jobs)):
            np.ascontiguousarray(arr).tofile(os.path.join(d, name + ".bin"))
        p = subprocess.run([NATIVE, d, str(calls)], capture_output=True, text=True, timeout=180)
        if p.returncode != 0:
            return {"error": f"exit {p.returncode}: {p.stderr.strip()[-300:]}"}
        return json.loads(p.stdout.strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001 (reported in the line, never fatal to the bench)
        return {"error": repr(e)[:300]}
    finally:
        shutil.rmtree(d, ignore_errors=True)


def config0_records_check(txs, inputs, gpu_records) -> dict:
    """configs[0]'s device-extracted records against the oracle
    (oracle/sighash_oracle.py: tx parse, txSigHash, decodeTxSig, HASH160
    template check) byte for byte — a parity check, not a CPU rate: the
    Python restatement's speed says nothing about haskoin-core's sighash, so
    it is not timed."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sighash_oracle as sh
    parsed = [sh.tx_parse(t) for t in txs]
    exp = b"".join(sh.std_input_record(parsed[t], i, p, val) for (t, i, p, val) in inputs)
    got = gpu_records.tobytes()
    n = len(inputs)
    rec_mism = sum(got[k * 168:(k + 1) * 168] != exp[k * 168:(k + 1) * 168] for k in range(n))
    msg_mism = sum(got[k * 168:k * 168 + 32] != exp[k * 168:k * 168 + 32] for k in range(n))
    return {"inputs": n, "record_mismatches_vs_oracle": int(rec_mism), "msg32_mismatches_vs_oracle": int(msg_mism),
            "checker": "oracle/sighash_oracle.py"}


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


def inproc_leg(v, torch, n: int, steps: int) -> dict:
    """The multi-device path the Haskell binding uses: ONE
    process opens every visible GPU through hkv_open(0, ...) and verifies
    BASELINE configs[4]'s 16,777,216-record batch from one pinned host batch
    with hkv_verify — contiguous 64-aligned shards per device, H2D pipelined
    with the verify on each device, verdict words merged on the host (D2H, no
    RCCL inside libhkv). PCIe-inclusive; checked against the construction
    labels. On one GPU it is the N = 1 point of that path."""
    import numpy as np
    import hkv
    # the records and labels on device 0 of the bench's own context, then to
    # the pinned batch of the all-device context
    recs = torch.empty(n * 168, dtype=torch.uint8, device="cuda")
    labels = torch.zeros((n + 63) // 64 * 2, dtype=torch.int32, device="cuda")
    v.gen_batch_device(0, CONFIG4_SEED, 0, n, POOL, UNC_PERMILLE, CONFIG4_INVALID_PERMILLE, recs.data_ptr(),
                       labels.data_ptr(), 0)
    torch.cuda.synchronize()
    host = recs.cpu().numpy()
    lab = labels.cpu().numpy().view(np.uint32)[: (n + 31) // 32].copy()
    del recs, labels
    torch.cuda.empty_cache()
    va = hkv.Verifier(hkv.VerifierConfig(device_ids=None, flags=1))
    try:
        nd = va.lib.hkv_ctx_num_devices(va.ctx)
        b = ctypes.c_void_p()
        rc = va.lib.hkv_batch_alloc(va.ctx, n, ctypes.byref(b))
        if rc != 0:
            return {"error": rc}
        try:
            ctypes.memmove(va.lib.hkv_batch_records(b), host.ctypes.data, n * 168)
            del host
            words = np.zeros((n + 31) // 32, dtype=np.uint32)
            wp = words.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
            rc = va.lib.hkv_verify(va.ctx, b, n, 0, wp)  # warm-up (allocations)
            if rc != 0:
                return {"error": rc}
            k = max(2, steps // 5)
            t0 = time.perf_counter()
            for _ in range(k):
                va.lib.hkv_verify(va.ctx, b, n, 0, wp)
            dt = (time.perf_counter() - t0) / k
            last = (n % 32) and ((1 << (n % 32)) - 1)
            diff = words ^ lab
            if last:
                diff[-1] &= last
            mism = int(np.unpackbits(diff.view(np.uint8)).sum())
            return {"devices": nd, "records": n, "ms": round(dt * 1e3, 2), "verifies_per_s": round(n / dt, 1),
                    "mismatches_vs_labels": mism, "accepted": int(np.unpackbits(words.view(np.uint8)).sum()),
                    "h2d_bytes": n * 168,
                    "workload": "BASELINE configs[4] batch (16,777,216 records, 5% invalid) from one pinned host "
                                "batch: hkv_open(all visible GPUs) + hkv_verify, PCIe-inclusive, verdict words "
                                "merged on the host"}
        finally:
            va.lib.hkv_batch_free(b)
    finally:
        va.close()


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


def adversarial_mix(v, torch, n: int, sptr: int, steps: int):
    """BASELINE configs[3]: 1,048,576 generated records (seed 0x484B5634), 30%
    of them mutated evenly into every invalid class of hkv/adversarial.py and
    5% into its special valid classes (labels fixed by construction, checked
    against the C restatement and OpenSSL in the tests and in the CPU leg
    here); verified in both modes; mismatches vs the labels must be 0."""
    import numpy as np
    from hkv import adversarial
    seed = 0x484B5634
    d = torch.empty(n * 168, dtype=torch.uint8, device="cuda")
    v.gen_records_device(0, seed, n, POOL, UNC_PERMILLE, d.data_ptr(), sptr)
    t = torch.empty(n * 168, dtype=torch.uint8, device="cuda")
    v.gen_records_device(0, seed, n, POOL, 1000, t.data_ptr(), sptr)  # same records, 65-byte keys (y source)
    torch.cuda.synchronize()
    adv, lab_lib, lab_hask, cls = adversarial.mutate(d.cpu().numpy(), seed=seed, twin=t.cpu().numpy())
    del t
    d.copy_(torch.from_numpy(adv))
    words = torch.zeros((n + 63) // 64 * 2, dtype=torch.int32, device=d.device)
    stream = torch.cuda.current_stream()
    out = {"records": n, "invalid_frac": round(float(np.isin(cls, np.arange(len(adversarial.INVALID_CLASSES))).mean()), 4),
           "special_valid_frac": round(float((cls >= len(adversarial.INVALID_CLASSES)).mean()), 4)}
    verdicts = {}
    for name, mode, lab in (("libsecp", 0, lab_lib), ("haskoin", 1, lab_hask)):
        v.verify_device(0, d.data_ptr(), n, mode, words.data_ptr(), sptr)
        torch.cuda.synchronize()
        got = adversarial.unpack_bits(words.cpu().numpy().view(np.uint32), n)
        verdicts[mode] = got
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        k = max(3, steps // 2)
        e0.record(stream)
        for _ in range(k):
            v.verify_device(0, d.data_ptr(), n, mode, words.data_ptr(), sptr)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / k
        out[name] = {"mismatches_vs_labels": int((got != lab).sum()), "accepts": int(got.sum()),
                     "ms": round(ms, 4), "verifies_per_s": round(n / (ms * 1e-3), 1)}
    out["workload"] = ("BASELINE configs[3]: 30% invalid, evenly: " + ", ".join(
        c for c, _, _ in adversarial.INVALID_CLASSES) + "; 5% special valid: reencode, valid_hybrid, r+n branch, "
        "edge u1/u2, u1=0, msg32>=n, ladder collisions; labels by construction")
    return out, adv, verdicts


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
                       "txids resident in HBM; <= n_cu blocks: 8 subtree workgroups per block + a top join, "
                       "more: one workgroup per block")
    return out


def load_traffic(path: str, n: int):
    """HBM bytes per ecmult launch from the committed PMC summary
    (tools/pmc_summary.py): FETCH_SIZE x 2 (MI355X_MICROARCH.md: on gfx950
    FETCH_SIZE reports 1/2 of the bytes of wide reads) + WRITE_SIZE, both KB
    counters x 1024, separate --pmc passes of the same 1M-record launch."""
    if not os.path.exists(path):
        return None, None
    try:
        tj = json.load(open(path))
    except Exception:
        return None, None
    if tj.get("per_verify_records") != n:
        return None, None
    f, w = tj.get("fetch_bytes_per_launch"), tj.get("write_bytes_per_launch")
    if f is None or w is None:
        return None, None
    raw = {"fetch_size_bytes": f, "write_size_bytes": w, "source": tj.get("source")}
    # VALU busy, occupancy and the integer instruction counts of
    # the same profiled launch
    for k in ("valu_busy_pct", "waves_per_simd", "SQ_INSTS_VALU", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64"):
        if k in tj:
            raw[k] = tj[k]
    return 2 * f + w, raw


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_devices() -> int:
    """GPUs this process may use, counted without HIP (the launcher parent
    starts the ranks by fork + exec and must not have touched the GPU first):
    the KFD topology's GPU nodes (non-zero gpu_id) whose render node this
    process can open (a device cgroup refuses the others), then the
    ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES filters."""
    import glob
    n = 0
    for node in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*")):
        try:
            if int(open(os.path.join(node, "gpu_id")).read().strip() or 0) == 0:
                continue
            minor = None
            for line in open(os.path.join(node, "properties")):
                k, _, val = line.partition(" ")
                if k == "drm_render_minor":
                    minor = int(val)
            if minor is None:
                continue
            fd = os.open(f"/dev/dri/renderD{minor}", os.O_RDWR | os.O_CLOEXEC)
            os.close(fd)
            n += 1
        except (OSError, ValueError):
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        val = os.environ.get(var)
        if val is not None:
            n = min(n, len([x for x in val.split(",") if x.strip()]))
    return n


def spawn_ranks(n: int, argv: list, mock: bool = False, share_device: bool = False) -> int:
    """`python bench.py --gpus N` without a launcher: start N rank processes
    (fresh interpreters, never an exec of this one) with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* set as torchrun would, wait for all of them and
    return the first non-zero exit code (the others are then killed by PID).
    Rank 0 prints the JSON line on the inherited stdout. The parent makes no
    GPU call; it fails fast when fewer than N devices are visible."""
    import subprocess
    if not mock:
        have = visible_devices()
        if (1 if share_device else n) > have:
            print(f"bench.py: --gpus {n} but only {have} GPU(s) visible", file=sys.stderr, flush=True)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HKV_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"bench.py: rank process {p.pid} exited with {code}; stopping the others", file=sys.stderr,
                      flush=True)
                for q in live:
                    q.kill()
        time.sleep(0.05)
    return rc


def mock_pattern(k):
    """Verdict of global record k in the CPU mock leg (a fixed bit pattern:
    the launcher test checks the gathered bitmap against it)."""
    import numpy as np
    k = np.asarray(k, dtype=np.uint64)
    return ((k * np.uint64(2654435761)) >> np.uint64(7)) & np.uint64(1)


def mock_main(args, world: int, rank: int) -> None:
    """The launcher and the multi-rank step on CPU (gloo): the same
    ShardedVerify, barrier, timing and max-over-ranks reduction as the GPU
    run, with a pattern writer instead of hkv_verify_device. For tests only
    (`--mock-cpu`); it prints a line marked "mock": true."""
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "haskoin-node_amd"))
    from hkv.records import bits_from_bools
    from hkv.shard import ShardedVerify
    use_dist = world > 1 or args.force_collective
    if use_dist:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("gloo")
    if os.environ.get("HKV_MOCK_FAIL_RANK") == str(rank):
        sys.exit(3)  # test hook: this rank dies inside the group, the others block in the all-gather
    n_total = args.config4_n

    def verify(lo, hi, bits):
        w = bits_from_bools(mock_pattern(np.arange(lo, hi)).astype(bool))
        bits.zero_()
        bits[: len(w)] = torch.from_numpy(w.view(np.int32))

    sv = ShardedVerify(torch, n_total, rank, world, verify, dist=dist if use_dist else None, device="cpu",
                       force_collective=use_dist)
    for _ in range(args.warmup):
        sv.step()
    if use_dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sv.step()
    if use_dist:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if use_dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    full = sv.bitmap()
    lab = bits_from_bools(mock_pattern(np.arange(sv.lo, sv.hi)).astype(bool))
    chk = torch.tensor([sv.slice_mismatches(full, lab)], dtype=torch.int64)
    devs = [{"rank": rank, "device": "cpu", "pid": os.getpid()}]
    if use_dist:
        dist.all_reduce(chk, op=dist.ReduceOp.SUM)
        gathered = [None] * world
        dist.all_gather_object(gathered, devs[0])
        devs = gathered
    if rank == 0:
        dt = t.item()
        print(json.dumps({"metric": "mock", "mock": True, "value": round(n_total * args.steps / dt, 1),
                          "n_gpus": world, "ranks_seen": world, "rank_devices": devs, "steps": args.steps,
                          "warmup": args.warmup, "mismatches": int(chk.item()), "global_batch": n_total,
                          "collective": "gloo" if use_dist else None,
                          "gather_vs_local_mismatches": sv.slice_mismatches(full, sv.local_bitmap())}),
              flush=True)
    if use_dist:
        dist.destroy_process_group()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one rank each). Without a launcher (WORLD_SIZE unset) N > 1 starts N rank processes; "
                         "under torchrun it must equal WORLD_SIZE")
    ap.add_argument("--mock-cpu", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--per-gpu", type=int, default=PER_GPU)
    ap.add_argument("--mode", type=int, default=0, help="0 = HKV_LIBSECP, 1 = HKV_HASKOIN")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-block-mix", action="store_true")
    ap.add_argument("--no-config0", action="store_true")
    ap.add_argument("--no-adversarial", action="store_true")
    ap.add_argument("--no-headers", action="store_true")
    ap.add_argument("--no-merkle", action="store_true")
    ap.add_argument("--no-host-path", action="store_true")
    ap.add_argument("--no-inproc", action="store_true",
                    help="skip the in-process all-GPU leg (hkv_open over every visible GPU, configs[4] from a pinned "
                         "host batch)")
    ap.add_argument("--config4", action="store_true",
                    help="BASELINE configs[4] (16,777,216 records, 5%% invalid, seed 0x484B5635, sharded over the "
                         "ranks); the default whenever WORLD_SIZE > 1")
    ap.add_argument("--config4-n", type=int, default=CONFIG4_N, help=argparse.SUPPRESS)
    ap.add_argument("--share-device", action="store_true",
                    help="test only: every rank runs on device 0 (the N > 1 code path on a 1-GPU lease); the "
                         "verdict words are all-gathered over gloo through host memory, since RCCL takes one rank "
                         "per GPU. Not a scaling measurement")
    ap.add_argument("--force-collective", action="store_true",
                    help="test only: at WORLD_SIZE 1 still create the nccl (RCCL) group with device_id and run the "
                         "step's all-gather of the verdict words on the device, on the stream libhkv enqueued on "
                         "(the N > 1 collective path on a 1-GPU lease)")
    ap.add_argument("--std-ibd", type=int, default=0, metavar="N_TX",
                    help="block_mix also times one N_TX-tx verifyStdInput batch (e.g. 560000: ~1M inputs)")
    ap.add_argument("--no-checker", action="store_true",
                    help="skip re-verifying every record of the slice on the host with oracle/secp_fast.c "
                         "(mismatches_vs_checker; outside the timed region)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "latest_pmc_traffic.json"))
    args = ap.parse_args()

    launched = "WORLD_SIZE" in os.environ
    if not launched and (args.gpus or 1) > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:], mock=args.mock_cpu, share_device=args.share_device))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr,
              flush=True)
        sys.exit(2)
    if args.mock_cpu:
        mock_main(args, world, rank)
        return

    import numpy as np
    import torch
    import torch.distributed as dist

    share = args.share_device
    gpu = 0 if share else local  # (--share-device: every rank on device 0)
    have = torch.cuda.device_count()
    if gpu >= have:
        print(f"bench.py: rank {rank} needs GPU {gpu} but only {have} visible", file=sys.stderr, flush=True)
        sys.exit(2)
    torch.cuda.set_device(gpu)
    # the group: N > 1 ranks, or --force-collective at N = 1 (a one-rank RCCL
    # group, so the device-side all-gather of the N > 1 step runs on one GPU)
    use_dist = world > 1 or (args.force_collective and not share)
    collective = None
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if share:
            dist.init_process_group("gloo")
            collective = "gloo"
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
            collective = "rccl" if torch.version.hip else "nccl"
    # the tensors the ranks reduce over: on the device for RCCL, in host
    # memory for gloo
    red_dev = "cpu" if share else "cuda"

    import hkv
    from hkv import opcount
    from hkv.shard import ShardedVerify

    # configs[1] (the N = 1 headline): 1M valid records per GPU, weak scaling.
    # configs[4] (every N > 1 run, or --config4): ONE global batch of 16M
    # records (5% invalid) sharded over the ranks, strong scaling.
    config4 = args.config4 or world > 1
    if config4:
        n_total, seed, inv = args.config4_n, CONFIG4_SEED, CONFIG4_INVALID_PERMILLE
    else:
        n_total, seed, inv = args.per_gpu * world, SEED, 0
    v = hkv.Verifier(hkv.VerifierConfig(device_ids=[gpu]))
    # a real (non-null) stream made current: libhkv enqueues on it and the RCCL
    # all-gather, which waits on torch's current stream, is ordered after the
    # verify (the null stream would not order against libhkv's own stream)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream

    def verify_shard(lo, hi, bits):
        v.verify_device(0, recs.data_ptr(), hi - lo, args.mode, bits.data_ptr(), sptr)

    sv = ShardedVerify(torch, n_total, rank, world, verify_shard, dist=dist if use_dist else None,
                       gather_on_host=share, force_collective=use_dist)
    n = sv.local_n
    recs = torch.empty(n * 168, dtype=torch.uint8, device="cuda")
    labels = torch.zeros((n + 63) // 64 * 2, dtype=torch.int32, device="cuda")
    # each rank generates exactly records [lo, hi) of the one global batch
    # (record k depends on (seed, k) only; hkv_gen_batch_device) with their
    # construction labels
    v.gen_batch_device(0, seed, sv.lo, n, POOL, UNC_PERMILLE, inv, recs.data_ptr(), labels.data_ptr(), sptr)
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        sv.step()
    torch.cuda.synchronize()
    v.lib.hkv_profile_enable(v.ctx, 1)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sv.step()
    torch.cuda.synchronize()
    if use_dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    pm, em, nl = ctypes.c_double(), ctypes.c_double(), ctypes.c_uint64()
    v.lib.hkv_profile_read(v.ctx, 0, ctypes.byref(pm), ctypes.byref(em), ctypes.byref(nl))
    sclk = ctypes.c_double()
    v.lib.hkv_profile_clock(v.ctx, 0, ctypes.byref(sclk))
    v.lib.hkv_profile_enable(v.ctx, 0)

    t = torch.tensor([dt, em.value / max(1, nl.value), pm.value / max(1, nl.value)], dtype=torch.float64,
                     device=red_dev)
    if use_dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt_max, ecm_ms, pro_ms = t.tolist()

    # self-check of the gathered bitmap: every rank compares its slice of the
    # assembled global bitmap with its construction labels; the counts are
    # summed over the ranks (outside the timed region), so every bit of the
    # gathered bitmap is checked against the label of the same global record
    full = sv.bitmap()
    lab_np = labels.cpu().numpy().view(np.uint32)
    # and the gathered bitmap's slice against the rank's own words as the
    # verify wrote them (before the collective): a gather that lost, moved
    # or raced a word shows here even where the labels would not
    own = sv.local_bitmap()
    chk = torch.tensor([sv.slice_mismatches(full, lab_np),
                        int(np.unpackbits(full.view(np.uint8), bitorder="little")[sv.lo:sv.hi].sum()),
                        int(np.unpackbits(lab_np.view(np.uint8), bitorder="little")[:n].sum()),
                        sv.slice_mismatches(full, own)],
                       dtype=torch.int64, device=red_dev)
    if use_dist:
        dist.all_reduce(chk, op=dist.ReduceOp.SUM)
    mismatches, accepted, label_valid, gather_vs_local = chk.tolist()
    # the same slice against the CPU checker, every record (summed over ranks)
    chkr = None
    if not args.no_checker:
        mine = np.unpackbits(full.view(np.uint8), bitorder="little")[sv.lo:sv.hi].astype(bool)
        chkr = checker_leg(recs.cpu().numpy(), mine, args.mode)
        ct = torch.tensor([chkr["checked"], -1 if chkr["mismatches"] is None else chkr["mismatches"],
                           chkr.get("seconds", 0.0) * 1000], dtype=torch.int64, device=red_dev)
        if use_dist:
            dist.all_reduce(ct, op=dist.ReduceOp.SUM)
        checked_all, mism_all, ms_all = ct.tolist()
        chkr = {"checked": checked_all,
                "mismatches": mism_all if chkr["mismatches"] is not None and mism_all >= 0 else None,
                "checker": chkr.get("checker"), "threads_rank0": chkr.get("threads"),
                "seconds_rank0": chkr.get("seconds"), "note": chkr.get("note")}
    import hashlib
    bitmap_sha = hashlib.sha256(full[: (n_total + 31) // 32].tobytes()).hexdigest()[:32]
    # which device every rank ran on (the line proves N ranks on N GPUs)
    props = torch.cuda.get_device_properties(gpu)
    me = {"rank": rank, "local_rank": local, "device": torch.cuda.current_device(), "name": props.name,
          "pci_bus_id": getattr(props, "pci_bus_id", None), "pci_device_id": getattr(props, "pci_device_id", None),
          "uuid": str(getattr(props, "uuid", "")) or None, "pid": os.getpid(), "local_n": n}
    rank_devices = [me]
    ranks_seen = 1
    if use_dist:
        ranks_seen = dist.get_world_size()
        rank_devices = [None] * world
        dist.all_gather_object(rank_devices, me)

    if rank == 0:
        value = n_total * args.steps / dt_max
        per_launch = n
        achieved = opcount.P_ALG_ECMULT * per_launch / (ecm_ms * 1e-3) / 1e12
        achieved_impl = opcount.ECMULT_PRODUCTS_PER_VERIFY * per_launch / (ecm_ms * 1e-3) / 1e12
        peak = opcount.PEAK_PRODUCTS_PER_S / 1e12
        f_mhz = sclk.value if 500.0 < sclk.value < 4000.0 else None
        peak_meas = opcount.R_MUL_MEASURED * opcount.N_CU * f_mhz * 1e6 / 1e12 if f_mhz else None
        traffic, traffic_raw = load_traffic(args.traffic_json, n)
        c0 = mix = hp = hdr = mkl = adv = None
        c0_recs = c0_got = c0_txs = c0_inputs = adv_recs = adv_got = None
        single = world == 1 and not config4  # the N = 1 headline run carries the other legs
        if single and not args.no_config0:
            c0, c0_recs, c0_got, c0_txs, c0_inputs = config0_block(v, torch, args.steps)
            c0["records_vs_oracle"] = config0_records_check(c0_txs, c0_inputs, c0_recs)
        if single and not args.no_block_mix:
            mix = block_mix(v, torch, args.steps, args.std_ibd)
        if single and not args.no_host_path:
            hp = host_path(v, recs, n, args.steps)
        if single and not args.no_headers:
            hdr = header_batches(v, torch, args.steps)
        if single and not args.no_merkle:
            mkl = merkle_batches(v, torch, args.steps)
        if single and not args.no_adversarial:
            adv, adv_recs, adv_got = adversarial_mix(v, torch, n, sptr, args.steps)
        inproc = None
        if single and not args.no_inproc:
            inproc = inproc_leg(v, torch, args.config4_n, args.steps)
        cpu = None
        if single and not args.no_cpu_baseline:
            samples = []
            if c0_recs is not None:
                samples.append(("config0_block", c0_recs, 1, c0_got))
            m2 = min(n, 16384)
            gpu2 = np.unpackbits(full[: (m2 + 31) // 32].view(np.uint8), bitorder="little")[:m2].astype(bool)
            samples.append(("config1_sample", recs[: m2 * 168].cpu().numpy(), args.mode, gpu2))
            if adv_recs is not None:
                m4 = min(n, 16384)
                for mode in (0, 1):
                    samples.append((f"config3_sample_{'libsecp' if mode == 0 else 'haskoin'}",
                                    adv_recs[: m4 * 168], mode, adv_got[mode][:m4]))
            cpu = cpu_baseline(samples, thread_sweep())
            # north_star: ">= 50x the all-core host libsecp256k1 verify rate"
            if cpu.get("value"):
                cpu["gpu_over_cpu"] = north_star_ratio(value, cpu)

        if config4:
            workload = (f"BASELINE configs[4]: one IBD-style batch of {n_total:,} records (configs[1] distribution "
                        f"plus {inv / 10:g}% invalid: flipped msg32 / r / s bit, another key, the negated key; "
                        f"seed 0x{seed:X}), contiguous 64-aligned shards, each rank generating only its slice; "
                        + ("one gloo all-gather of the verdict words through host memory per step (--share-device: "
                           "every rank on device 0; a test of the N > 1 code path, not a scaling point)" if share else
                           "one RCCL all-gather of the verdict bitmap per step" if collective == "rccl" else
                           "no collective (one rank; --force-collective runs the RCCL all-gather at N = 1)"))
        else:
            workload = ("BASELINE configs[1]: 1,048,576 valid (hash,r,s,pubkey) per GPU, 90% compressed / 10% "
                        "uncompressed keys, 65,536-key pool")
        line = {
            "metric": "ECDSA verifies/sec (1/8 GPU) + verdict mismatches vs libsecp256k1",
            "value": round(value, 1),
            "unit": "verifies/s",
            "n_gpus": world,
            "ranks_seen": ranks_seen,
            "rank_devices": rank_devices,
            "share_device": share,
            "collective": collective,
            "force_collective": bool(args.force_collective and world == 1 and not share),
            "gather_vs_local_mismatches": gather_vs_local,
            "bitmap_sha256_128": bitmap_sha,
            "bitmap_equals_1gpu": (bitmap_sha == CONFIG4_BITMAP_SHA)
                                  if (config4 and n_total == CONFIG4_N and seed == CONFIG4_SEED and args.mode == 0)
                                  else None,
            "launcher": ("bench.py spawn" if os.environ.get("HKV_BENCH_SPAWNED") else
                         "torchrun" if "TORCHELASTIC_RUN_ID" in os.environ or "GROUP_RANK" in os.environ else
                         "external" if world > 1 else "single process"),
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if config4 else "weak",
            "vs_baseline": None,
            "dtype": "u32 (256-bit integer limbs)",
            "data": "synthetic (keyless-constructed secp256k1 tuples generated on device; labels by construction)",
            "config": {"workload": workload,
                       "global_batch": n_total, "per_gpu": n, "mode": "LIBSECP" if args.mode == 0 else "HASKOIN",
                       "seed": seed, "invalid_permille": inv, "parallelism": f"dp{world}"},
            "mismatches": mismatches,
            "accepted": accepted,
            "label_valid": label_valid,
            "mismatches_note": "every bit of the (all-gathered) verdict bitmap vs the construction label of the "
                               "same global record, summed over ranks; every bit vs the libsecp256k1-class CPU "
                               "restatement: mismatches_vs_checker; GPU vs CPU implementations on the same "
                               "records: cpu_baseline.samples.*.*.mismatches_vs_gpu (N = 1)",
            "mismatches_vs_checker": chkr,
            "kernel_ms": {"prologue": round(pro_ms, 4), "ecmult": round(ecm_ms, 4)},
            "roofline": {"bound": "valu_int", "achieved": round(achieved, 4), "peak": round(peak, 3),
                         "unit": "T limb-products/s (v_mad_u64_u32)", "frac": round(achieved / peak, 4),
                         "traffic": traffic,
                         "kernel": "ecmult stage: hkv_ecmult_kernel (u2*Q on E_w) + hkv_finish_kernel (u1*G, "
                                   "num/den) + hkv_rare_kernel + hkv_yverdict_kernel (den^-1, y_c^2 == w)",
                         "p_alg": opcount.P_ALG_ECMULT,
                         "p_alg_note": "reference algorithm (libsecp256k1 ecmult: GLV + wNAF5 Q, w=15 G tables, "
                                       "129 doublings) priced in 32x32 limb products; frozen (hkv/opcount.py)",
                         "p_impl": opcount.ECMULT_PRODUCTS_PER_VERIFY,
                         "achieved_impl": round(achieved_impl, 4),
                         "frac_nominal": round(achieved / peak, 4),
                         "sclk_mhz": round(f_mhz, 1) if f_mhz else None,
                         "peak_measured_clock": round(peak_meas, 3) if peak_meas else None,
                         "frac_measured_clock": round(achieved / peak_meas, 4) if peak_meas else None,
                         "measured_rate_note": "57.07 lane-products/clk/CU (profiles/r01_ubench_int.json) x 256 "
                                               "CUs x the clock block 0 of the launch ran at (clock64/wall_clock64)",
                         "traffic_raw": traffic_raw,
                         "traffic_note": "HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE "
                                         "halving, MI355X_MICROARCH.md); algorithmic input = 168 B/verify"},
            "cpu_baseline": cpu,
            "config0": c0,
            "block_mix": mix,
            "adversarial": adv,
            "headers": hdr,
            "merkle": mkl,
            "host_path": hp,
            "inproc": inproc,
        }
        print(json.dumps(line), flush=True)
    v.close()
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
