"""The block paths alone, for a rocprofv3 kernel trace (profiles/r03_block_*):
BASELINE configs[0] (2,000 P2PKH txs) and configs[2] (2,000-tx P2PKH + P2WPKH
mix), each run K times through hkv_verify_std_inputs_device (the fused
small-batch kernel) and K times through hkv_std_inputs_device (extraction
only), on one stream, nothing else on the GPU.

    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o block -- python tools/block_trace.py
    python tools/block_trace.py --report gpurun_out/prof   (median launch per kernel and grid -> JSON)
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "haskoin-node_amd"))


def report(d: str) -> dict:
    import csv
    import glob
    import json
    import statistics
    from collections import defaultdict
    durs = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            grid = int(r['Grid_Size_X']) * int(r['Grid_Size_Y']) * int(r['Grid_Size_Z'])
            durs[f"{name}@grid{grid}"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {k: {"launches": len(v), "median_us": round(statistics.median(v), 1), "min_us": round(min(v), 1)}
           for k, v in sorted(durs.items())}
    json.dump(out, open(os.path.join(d, "kernel_by_grid.json"), "w"), indent=1)
    for k, v in out.items():
        print(f"{v['median_us']:9.1f} us  x{v['launches']:3d}  {k}")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--batch32", action="store_true", help="also the 64,000-tx batch (bench block_mix.batch32)")
    ap.add_argument("--report", default=None, help="summarise a rocprofv3 csv output directory")
    ap.add_argument("--stamps", action="store_true",
                    help="one profiled configs[0] call last: print its workgroups' raw start / end clock stamps "
                         "(s_memrealtime ticks) to set beside the trace's dispatch timestamps")
    a = ap.parse_args()
    if a.report:
        report(a.report)
        return
    import torch
    import hkv
    from hkv import blockgen
    v = hkv.Verifier(hkv.VerifierConfig(device_ids=[0]))
    st = torch.cuda.Stream()
    blocks = (("configs0", blockgen.make_p2pkh_block(v, torch)),
              ("configs2", blockgen.make_block(v, torch, n_tx=2000, seed=blockgen.SEED + 2000)))
    if a.batch32:
        blocks += (("batch32", blockgen.make_block(v, torch, n_tx=64000, seed=blockgen.SEED + 64000)),)
    for name, (txs, inputs) in blocks:
        db = blockgen.DeviceBlock(torch, txs, inputs)
        for what in ("verify", "extract"):
            for _ in range(a.k):
                if what == "verify":
                    v.verify_std_inputs_device(0, db.txs, db.d_jobs.data_ptr(), db.n, -1, db.records.data_ptr(),
                                               db.bits.data_ptr(), st.cuda_stream)
                else:
                    v.std_inputs_device(0, db.txs, db.d_jobs.data_ptr(), db.n, -1, db.records.data_ptr(),
                                        st.cuda_stream)
            torch.cuda.synchronize()
            print(name, what, db.n, flush=True)
        if a.stamps and name == "configs0":
            import ctypes
            v.lib.hkv_profile_enable(v.ctx, 1)
            v.verify_std_inputs_device(0, db.txs, db.d_jobs.data_ptr(), db.n, -1, db.records.data_ptr(),
                                       db.bits.data_ptr(), st.cuda_stream)
            torch.cuda.synchronize()
            ng = (db.n + 255) // 256 * 256 // 16
            g = (ctypes.c_uint64 * (2 * ng))()
            tick = ctypes.c_double()
            v.lib.hkv_profile_group_stamps(v.ctx, 0, g, ng, ctypes.byref(tick))
            v.lib.hkv_profile_enable(v.ctx, 0)
            starts, ends = [g[2 * k] for k in range(ng)], [g[2 * k + 1] for k in range(ng)]
            print("stamps", {"tick_ns": tick.value, "start_min": min(starts), "start_max": max(starts),
                             "end_min": min(ends), "end_max": max(ends)}, flush=True)
    v.close()


if __name__ == "__main__":
    main()
