"""Kernel timeline of the last full-grid standard-input call in a rocprofv3
kernel trace (tools/block_trace.py --batch32 under `rocprofv3 --kernel-trace
--output-format csv`): every hkv kernel from that call's tx index launch to
the launches after its mid-size ecmult, with start / end relative to the
first one — concurrent launches (the hash half on its own stream) show as
overlapping intervals. profiles/r04f/batch32_timelines.txt.

    python tools/trace_timeline.py gpurun_out/prof_x/b32_kernel_trace.csv
"""
import csv
import sys


def main(path: str) -> None:
    rows = [r for r in csv.DictReader(open(path)) if "hkv" in r["Kernel_Name"] and "gen_" not in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ec = [i for i, r in enumerate(rows) if "ecmult_kernel<true" in r["Kernel_Name"]]
    i = ec[-1]
    j = i  # back to the call's tx index / tx hash launch
    while j > 0 and not ("tx_hash" in rows[j]["Kernel_Name"] or "tx_index" in rows[j]["Kernel_Name"]):
        j -= 1
    while j > 0 and ("tx_index" in rows[j - 1]["Kernel_Name"] or "tx_hash" in rows[j - 1]["Kernel_Name"]):
        j -= 1
    t0 = int(rows[j]["Start_Timestamp"])
    for r in rows[j:i + 7]:
        nm = r["Kernel_Name"].split("(")[0].replace("void ", "")
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"])
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{nm[:40]:40s} grid {g:8d} start {(s - t0) / 1e3:8.1f} end {(e - t0) / 1e3:8.1f} dur {(e - s) / 1e3:8.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
