"""Summarise a tools/profile_round.sh output directory into profiles/.

    python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<tag>

Writes <dest>/kernel_stats.csv (rocprofv3 --kernel-trace --stats summary),
<dest>/pmc.json (per-kernel counters of the 1M-record bench dispatches) and
profiles/latest_pmc_traffic.json, which bench.py reads for roofline.traffic:
HBM-side bytes per ecmult launch = (FETCH_SIZE + WRITE_SIZE) * 1024, from
separate --pmc passes (MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KB
counted at the L2 memory side; Infinity-Cache hits are included). The raw
counters are stored; bench.py applies the guide's gfx950 read correction
(FETCH_SIZE reports 1/2 of the bytes of wide reads) as 2 x FETCH + WRITE.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


def kname(raw: str) -> str:
    """Kernel name without the namespace / argument list. The ecmult instances:
    round 4 hkv_ecmult_kernel<ILP, STDPRO> (-> "", _mid, _mid_std) and
    hkv_finish_kernel<ILP, LATE> (-> "", _mid, _late, _mid_late);
    round 3 hkv_ecmult_kernel<ILP> (<false> full grid, <true> -> _mid) and
    hkv_pair_split_kernel<STD> / hkv_block_kernel<STD> (<false> -> _rec,
    <true> -> _std); the round-2
    hkv_ecmult_kernel<SPLIT, ILP> names map as before (<false, false> full
    grid, <false, true> _mid, <true, *> _split)."""
    k = raw.split("(")[0].replace("hkv::", "")
    if k.startswith("void "):
        k = k[5:]
    # round 4: hkv_ecmult_kernel<ILP, STDPRO> and hkv_finish_kernel<ILP, LATE>
    if k.startswith("hkv_ecmult_kernel<") or k.startswith("hkv_finish_kernel<"):
        base, args = k.split("<", 1)
        flags = [a.strip() == "true" for a in args.rstrip(">").split(",")]
        if len(flags) == 2:
            second = "_std" if base == "hkv_ecmult_kernel" else "_late"
            return base + ("_mid" if flags[0] else "") + (second if flags[1] else "")
    k = k.replace("<false, false>", "").replace("<false, true>", "_mid")
    k = k.replace("<true, true>", "_split").replace("<true, false>", "_split")
    if k.startswith("hkv_pair_split_kernel") or k.startswith("hkv_block_kernel"):
        return k.replace("<false>", "_rec").replace("<true>", "_std")
    if k.startswith("hkv_ecmult_kernel"):
        return k.replace("<false>", "").replace("<true>", "_mid")
    return k.replace("<false>", "").replace("<true>", "_split")


def main(src: str, dst: str) -> None:
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(dst, "kernel_stats.csv"))
    # per (kernel, grid) launch durations from the kernel trace: the ecmult
    # grid is fixed (grid-stride), so the median is the 1M-record launch and
    # the open-time self-check launch does not skew it
    traces = glob.glob(os.path.join(src, "trace", "*kernel_trace.csv"))
    if traces:
        durs = defaultdict(list)
        for r in csv.DictReader(open(traces[0])):
            k = kname(r["Kernel_Name"])
            g = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
            durs[(k, g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        ks = {}
        for (k, g), v in sorted(durs.items()):
            v.sort()
            ks[f"{k}@grid{g}"] = {"calls": len(v), "avg_us": round(sum(v) / len(v), 2),
                                  "median_us": round(v[len(v) // 2], 2), "min_us": round(v[0], 2),
                                  "max_us": round(v[-1], 2)}
        json.dump(ks, open(os.path.join(dst, "kernel_by_grid.json"), "w"), indent=1)
    per = defaultdict(lambda: defaultdict(list))
    grid = {}
    for f in glob.glob(os.path.join(src, "pmc_*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            g = int(r["Grid_Size"])
            k = kname(r["Kernel_Name"])
            if g < 65536 or not k.startswith("hkv_"):
                continue
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            grid[k] = g
    out = {k: {c: sorted(v)[len(v) // 2] for c, v in d.items()} for k, d in per.items()}  # median launch
    for k in out:
        out[k]["Grid_Size"] = grid[k]
    json.dump(out, open(os.path.join(dst, "pmc.json"), "w"), indent=1)
    e = out.get("hkv_ecmult_kernel", {})
    if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
        t = {"kernel": "hkv_ecmult_kernel", "per_verify_records": 1 << 20,
             "fetch_bytes_per_launch": e["FETCH_SIZE"] * 1024, "write_bytes_per_launch": e["WRITE_SIZE"] * 1024,
             "hbm_bytes_per_launch": (e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024,
             "source": os.path.relpath(dst), "hbm_bytes_per_launch_corrected": (2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024,
             "note": "raw FETCH_SIZE / WRITE_SIZE (KB*1024), separate pmc passes; corrected = 2 x FETCH + WRITE"}
        # VALU busy and occupancy of the same launch. VALUBusy =
        # SQ_ACTIVE_INST_VALU x 4 cycles / (SIMDs x GRBM_GUI_ACTIVE per XCD);
        # the wave count over the SIMDs is the resident waves per SIMD (the
        # grid is sized to exactly one resident round: grid-stride)
        n_simd, n_xcd = 1024, 8
        if "SQ_ACTIVE_INST_VALU" in e and "GRBM_GUI_ACTIVE" in e:
            gui = e["GRBM_GUI_ACTIVE"] / n_xcd
            t["valu_busy_pct"] = round(100.0 * e["SQ_ACTIVE_INST_VALU"] * 4 / n_simd / gui, 1)
            t["grbm_gui_active_per_xcd"] = gui
        if "SQ_WAVES" in e:
            t["waves_per_simd"] = round(e["SQ_WAVES"] / n_simd, 2)
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64"):
            if c in e:
                t[c] = e[c]
        json.dump(t, open(os.path.join(os.path.dirname(dst.rstrip("/")), "latest_pmc_traffic.json"), "w"), indent=1)
    print(json.dumps({k: {c: "%.4g" % v for c, v in d.items()} for k, d in out.items()}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
