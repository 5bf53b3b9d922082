"""Kernel timeline of one configs[2] block verify (run under rocprofv3).

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tl -- \
        python3 tools/block_timeline.py
    python3 tools/block_timeline.py --report gpurun_out/tl

The run verifies the 2,000-tx block K times with a device sync between calls,
so each call's kernels form one group; --report prints the median start/end of
every kernel relative to the group's first kernel, and the gaps between them.
"""
import argparse
import glob
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "haskoin-node_amd"))


def run(k: int) -> None:
    import torch
    import hkv
    from hkv import blockgen
    v = hkv.Verifier(hkv.VerifierConfig(device_ids=[0]))
    txs, inputs = blockgen.make_block(v, torch, n_tx=2000, seed=blockgen.SEED + 2000)
    db = blockgen.DeviceBlock(torch, txs, inputs)
    st = torch.cuda.Stream()
    torch.cuda.synchronize()
    for _ in range(k):
        v.verify_std_inputs_device(0, db.txs, db.d_jobs.data_ptr(), db.n, -1, db.records.data_ptr(),
                                   db.bits.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
    print("done", k, "block verifies of", db.n, "inputs")


def report(d: str) -> None:
    import csv
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy:" + r.get("Direction", "?")))
    rows.sort()
    # groups: the verify calls start with hkv_tx_hash_kernel (index + BIP143 hashes)
    groups, cur = [], None
    for r in rows:
        if r[2].endswith("hkv_tx_hash_kernel"):
            cur = []
            groups.append(cur)
        if cur is not None:
            cur.append(r)
    groups = [g for g in groups[2:] if g]  # skip warm-up calls
    n = min(len(g) for g in groups)
    print(f"{len(groups)} block verifies, {n} ops each (median over calls, us from the first kernel's start)")
    t_end = []
    for i in range(n):
        s = statistics.median((g[i][0] - g[0][0]) / 1e3 for g in groups)
        e = statistics.median((g[i][1] - g[0][0]) / 1e3 for g in groups)
        gap = statistics.median(((g[i][0] - g[i - 1][1]) / 1e3 if i else 0.0) for g in groups)
        print(f"  {groups[0][i][2][:48]:48s} start {s:8.1f} end {e:8.1f} dur {e - s:7.1f} gap-before {gap:6.1f}")
        t_end.append(e)
    print(f"  span {max(t_end):.1f} us")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=12)
    ap.add_argument("--report", default=None)
    a = ap.parse_args()
    report(a.report) if a.report else run(a.k)
