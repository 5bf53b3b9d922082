"""One tip block as a node sees it: configs[0]'s block
verified by ONE hkv_verify_std_inputs_device call on an idle GPU, repeated,
with the GPU idle for a few ms before each call (a block arrives alone,
Node.hs:151-174). Per call: the host's enqueue time, the HIP-event latency
around the call, and — under a rocprofv3 kernel trace — each kernel's
duration and the gaps between them.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_iso -o iso -- python3 tools/isolated_call.py run gpurun_out/iso_host.json
    python3 tools/isolated_call.py report gpurun_out/prof_iso gpurun_out/iso_host.json
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "haskoin-node_amd"))


def run(out_json: str, calls: int = 40, idle_ms: float = 5.0) -> None:
    import torch
    import hkv
    from hkv import blockgen
    v = hkv.Verifier(hkv.VerifierConfig(device_ids=[0]))
    st = torch.cuda.Stream()
    txs, inputs = blockgen.make_p2pkh_block(v, torch)
    db = blockgen.DeviceBlock(torch, txs, inputs)

    def call():
        v.verify_std_inputs_device(0, db.txs, db.d_jobs.data_ptr(), db.n, -1, db.records.data_ptr(),
                                   db.bits.data_ptr(), st.cuda_stream)

    for _ in range(20):  # warm (allocations, code objects)
        call()
    torch.cuda.synchronize()
    rows = []
    for _ in range(calls):
        time.sleep(idle_ms * 1e-3)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter_ns()
        e0.record(st)
        t1 = time.perf_counter_ns()
        call()
        t2 = time.perf_counter_ns()
        e1.record(st)
        torch.cuda.synchronize()
        t3 = time.perf_counter_ns()
        rows.append({"event_us": e0.elapsed_time(e1) * 1e3, "enqueue_us": (t2 - t1) / 1e3,
                     "host_wall_us": (t3 - t0) / 1e3})
    json.dump({"calls": rows, "idle_ms": idle_ms, "inputs": db.n}, open(out_json, "w"))
    med = {k: round(statistics.median(r[k] for r in rows), 1) for k in rows[0]}
    print(json.dumps({"isolated_call_median": med}), flush=True)
    v.close()


def report(trace_dir: str, host_json: str) -> None:
    import csv
    import glob
    ks = []
    for f in glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    ks.sort()
    host = json.load(open(host_json))
    n = len(host["calls"])
    # the last n calls: (block kernel, tail kernel) pairs (or the block
    # kernel alone, for a build that runs the tail inside it)
    pairs = []
    i = len(ks) - 1
    while i >= 0 and len(pairs) < n:
        if i > 0 and "ms_tail" in ks[i][2] and "block_kernel" in ks[i - 1][2]:
            pairs.append((ks[i - 1], ks[i]))
            i -= 2
        elif "block_kernel" in ks[i][2]:
            pairs.append((ks[i], ks[i]))
            i -= 1
        else:
            i -= 1
    pairs.reverse()
    blk = [(b[1] - b[0]) / 1e3 for b, _ in pairs]
    tail = [(t[1] - t[0]) / 1e3 for b, t in pairs if t is not b]
    gap = [(t[0] - b[1]) / 1e3 for b, t in pairs if t is not b]
    span = [(t[1] - b[0]) / 1e3 for b, t in pairs]
    ev = [r["event_us"] for r in host["calls"]]
    enq = [r["enqueue_us"] for r in host["calls"]]
    med = lambda x: round(statistics.median(x), 1) if x else None
    out = {"calls": len(pairs), "idle_ms_before_each": host["idle_ms"],
           "event_latency_us": med(ev), "host_enqueue_us": med(enq),
           "block_kernel_us": med(blk), "gap_block_to_tail_us": med(gap), "tail_kernel_us": med(tail),
           "block_start_to_tail_end_us": med(span),
           "outside_kernels_us": round(med(ev) - med(span), 1) if pairs else None,
           "note": "event latency = HIP events on the call's stream around one call after >= idle_ms of GPU idle; "
                   "outside_kernels = that latency minus the block kernel's start to the tail kernel's end (host "
                   "enqueue before the first dispatch, dispatch, the event records)"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        report(sys.argv[2], sys.argv[3])
