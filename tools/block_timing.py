"""Timing probe for the configs[0] block call (round 4): the bench's
`config0.total_us` (HIP events around k back-to-back calls) reads ~267 us
while `back_to_back32` (host clock around 32 back-to-back calls) reads
~256 us per block. This times the same call several ways, in alternation, so
the difference can be attributed: events around k = 3 / 10 / 32 calls, the host
clock around 32 calls, events around each call alone, and the same with the
events on a stream that has not been idle.

    python tools/block_timing.py > gpurun_out/block_timing.txt   (configs[0], then the 64,000-tx batch)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "haskoin-node_amd"))


def main():
    import torch
    import hkv
    from hkv import blockgen
    v = hkv.Verifier(hkv.VerifierConfig(device_ids=[0]))
    st = torch.cuda.Stream()
    out = {}
    for label in ("configs0", "batch32"):
        if label == "configs0":
            txs, inputs = blockgen.make_p2pkh_block(v, torch)
        else:
            txs, inputs = blockgen.make_block(v, torch, n_tx=64000, seed=blockgen.SEED + 64000)
        out[label] = probe(v, torch, st, blockgen.DeviceBlock(torch, txs, inputs))
        print(json.dumps({label: out[label]}), flush=True)
    v.close()


def probe(v, torch, st, db):

    def run():
        v.verify_std_inputs_device(0, db.txs, db.d_jobs.data_ptr(), db.n, -1, db.records.data_ptr(),
                                   db.bits.data_ptr(), st.cuda_stream)

    for _ in range(20):
        run()
    torch.cuda.synchronize()

    def events(k):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(k):
            run()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / k

    def events_busy(k):
        # the stream is already busy with 4 calls when e0 is recorded
        torch.cuda.synchronize()
        for _ in range(4):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(k):
            run()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / k

    def host(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            run()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6 / k

    def enqueue(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            run()
        t = (time.perf_counter() - t0) * 1e6 / k
        torch.cuda.synchronize()
        return t

    res = {}
    for rep in range(3):
        for name, fn in (("events_k3", lambda: events(3)), ("events_k10", lambda: events(10)),
                         ("events_k32", lambda: events(32)), ("events_busy_k10", lambda: events_busy(10)),
                         ("host_k32", lambda: host(32)), ("host_k10", lambda: host(10)),
                         ("events_k1", lambda: events(1)), ("enqueue_k32", lambda: enqueue(32))):
            res.setdefault(name, []).append(round(fn(), 1))
    return {"inputs": db.n, "us_per_call": res}


if __name__ == "__main__":
    main()
