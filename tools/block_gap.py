"""Where the block kernel's launch time goes outside its workgroups (round 4).

rocprofv3 puts hkv_block_kernel<true> at ~252 us on a configs[0] block while
its workgroups' own start / end stamps span ~236 us. This runs profiled
configs[0] calls bracketed by a one-thread marker kernel that writes the same
100-MHz wall clock (tools/stamp_marker.hip), so under a kernel trace each
call's workgroup stamps can be placed on the trace's time axis:

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_gap -o gap -- python3 tools/block_gap.py run
    python3 tools/block_gap.py report gpurun_out/prof_gap/gap_kernel_trace.csv gpurun_out/block_gap_stamps.json
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "haskoin-node_amd"))


def run(out_json: str) -> None:
    import torch
    import hkv
    from hkv import blockgen
    mk = ctypes.CDLL(os.path.join(ROOT, "tools", "libstampmarker.so"))
    v = hkv.Verifier(hkv.VerifierConfig(device_ids=[0]))
    st = torch.cuda.Stream()
    txs, inputs = blockgen.make_p2pkh_block(v, torch)
    db = blockgen.DeviceBlock(torch, txs, inputs)

    def call():
        v.verify_std_inputs_device(0, db.txs, db.d_jobs.data_ptr(), db.n, -1, db.records.data_ptr(),
                                   db.bits.data_ptr(), st.cuda_stream)

    for _ in range(10):
        call()
    torch.cuda.synchronize()
    m = torch.zeros(2, dtype=torch.int64, device="cuda")
    ng = (db.n + 255) // 256 * 256 // 16
    res = []
    v.lib.hkv_profile_enable(v.ctx, 1)
    for _ in range(5):
        mk.stamp_marker(ctypes.c_void_p(m.data_ptr()), 0, ctypes.c_void_p(st.cuda_stream))
        call()
        mk.stamp_marker(ctypes.c_void_p(m.data_ptr()), 1, ctypes.c_void_p(st.cuda_stream))
        torch.cuda.synchronize()
        g = (ctypes.c_uint64 * (2 * ng))()
        tick = ctypes.c_double()
        v.lib.hkv_profile_group_stamps(v.ctx, 0, g, ng, ctypes.byref(tick))
        mm = m.cpu().tolist()
        res.append({"marker0": mm[0], "marker1": mm[1], "tick_ns": tick.value,
                    "start_min": min(g[2 * k] for k in range(ng)), "start_max": max(g[2 * k] for k in range(ng)),
                    "end_max": max(g[2 * k + 1] for k in range(ng)),
                    "starts": [g[2 * k] for k in range(ng)], "ends": [g[2 * k + 1] for k in range(ng)]})
    v.lib.hkv_profile_enable(v.ctx, 0)
    json.dump(res, open(out_json, "w"), indent=1)
    v.close()


def report(trace_csv: str, stamps_json: str) -> None:
    import csv
    rows = [r for r in csv.DictReader(open(trace_csv)) if "hkv" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    calls = []
    for k, r in enumerate(rows):
        if "stamp_marker" in r["Kernel_Name"] and k + 4 < len(rows) and "stamp_marker" in rows[k + 4]["Kernel_Name"]:
            calls.append(rows[k:k + 5])
    stamps = json.load(open(stamps_json))
    for c, s in zip(calls[-len(stamps):], stamps):
        t = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in c]
        tick_ns = s["tick_ns"]
        # tick -> trace ns from the two markers (each tick lies inside its marker's interval)
        off0 = (t[0][0] + t[0][1]) / 2 - s["marker0"] * tick_ns
        off1 = (t[4][0] + t[4][1]) / 2 - s["marker1"] * tick_ns
        off = (off0 + off1) / 2
        b0, b1 = t[2]
        ws, we = s["start_min"] * tick_ns + off, s["end_max"] * tick_ns + off
        print(json.dumps({"index_us": round((t[1][1] - t[1][0]) / 1e3, 2), "block_us": round((b1 - b0) / 1e3, 2),
                          "tail_us": round((t[3][1] - t[3][0]) / 1e3, 2),
                          "block_start_to_first_group_us": round((ws - b0) / 1e3, 2),
                          "groups_span_us": round((we - ws) / 1e3, 2),
                          "last_group_to_block_end_us": round((b1 - we) / 1e3, 2),
                          "marker_fit_disagreement_us": round((off1 - off0) / 1e3, 2)}))


def groups(stamps_json: str) -> None:
    """Each call's workgroup end times (us after the call's first start) by
    XCD (blockIdx % 8) and the slowest groups."""
    import statistics
    for s in json.load(open(stamps_json)):
        t0, us = min(s["starts"]), s["tick_ns"] * 1e-3
        ends = [(e - t0) * us for e in s["ends"]]
        by = {x: [ends[b] for b in range(len(ends)) if b % 8 == x and ends[b] - (s["starts"][b] - t0) * us > 200]
              for x in range(8)}
        slow = sorted(range(len(ends)), key=lambda b: -ends[b])[:8]
        print(json.dumps({"median_by_xcd": {x: round(statistics.median(v), 1) for x, v in by.items() if v},
                          "max_by_xcd": {x: round(max(v), 1) for x, v in by.items() if v},
                          "slowest": [(b, round(ends[b], 1)) for b in slow]}))


if __name__ == "__main__":
    if sys.argv[1] == "groups":
        groups(sys.argv[2])
    elif sys.argv[1] == "run":
        run(sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "block_gap_stamps.json"))
    else:
        report(sys.argv[2], sys.argv[3])
