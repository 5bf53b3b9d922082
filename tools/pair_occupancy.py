"""The pair kernel's per-batch time against its workgroups per CU: blocks of
configs[2]'s mix at 4,500 / 9,000 / 13,500 txs (about 1, 2 and 3 workgroups
of 32 inputs per CU on 256 CUs), HBM-resident, verified end to end
(bench.py _time_block). Prints one JSON line per size.

    python3 tools/pair_occupancy.py > gpurun_out/pair_occ.jsonl
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "haskoin-node_amd"))


def main() -> None:
    import torch
    import hkv
    import bench
    from hkv import blockgen
    v = hkv.Verifier(hkv.VerifierConfig(device_ids=[0]))
    st = torch.cuda.Stream()
    for n_tx in (4500, 9000, 13500):
        txs, inputs = blockgen.make_block(v, torch, n_tx=n_tx, seed=blockgen.SEED + n_tx)
        db = blockgen.DeviceBlock(torch, txs, inputs)
        res, _ = bench._time_block(v, torch, db, st, 10)
        print(json.dumps({"txs": n_tx, "inputs": res["inputs"], "workgroups": (res["inputs"] + 31) // 32,
                          "total_us": res["total_us"], "reps": res["total_us_reps"], "rejected": res["rejected"],
                          "latency_us": res["latency_us"]}), flush=True)
    v.close()


if __name__ == "__main__":
    main()
