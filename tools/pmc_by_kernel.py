"""Median per-dispatch PMC values by kernel from rocprofv3 counter_collection CSVs.

    python3 tools/pmc_by_kernel.py gpurun_out/<dir> [kernel-substring ...]
"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def main() -> None:
    d = sys.argv[1]
    pick = sys.argv[2:]
    vals = defaultdict(lambda: defaultdict(dict))  # kernel -> counter -> dispatch -> value
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if pick and not any(p in k for p in pick):
                continue
            disp = (f, r.get("Dispatch_Id", r.get("Correlation_Id", "")))
            vals[k][r["Counter_Name"]][disp] = vals[k][r["Counter_Name"]].get(disp, 0.0) + float(r["Counter_Value"])
    for k, cs in sorted(vals.items()):
        print(k)
        for c, dv in sorted(cs.items()):
            print(f"  {c:24s} {statistics.median(dv.values()):16.1f}  ({len(dv)} dispatches)")


if __name__ == "__main__":
    main()
