"""Mean counter value per dispatch of each (kernel, grid) in rocprofv3 --pmc
output directories: the per-launch FETCH_SIZE / WRITE_SIZE (KB) of the 1M
ecmult and finish launches, and the corrected HBM bytes per launch
(2 x FETCH + WRITE, the gfx950 read correction of MI355X_MICROARCH.md).

    python tools/pmc_kernel_bytes.py DIR [DIR ...]"""
import collections
import csv
import glob
import os
import sys


def load(d):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0].replace("hkv::", "").replace("void ", "")
            acc[(k, int(row["Grid_Size"]), row["Counter_Name"])].append(float(row["Counter_Value"]))
    return acc


def main(dirs):
    for d in dirs:
        acc = load(d)
        print(f"== {d}")
        for (k, g, c), v in sorted(acc.items()):
            if ("ecmult" in k or "finish" in k) and g >= 65536:
                print(f"  {k:40s} grid {g:8d} {c:12s} dispatches {len(v):3d} mean {sum(v) / len(v):14.1f} KB "
                      f"({sum(v) / len(v) * 1024 / 1e9:.3f} GB)")


if __name__ == "__main__":
    main(sys.argv[1:])
