"""Experiment: std-input extraction time for a config-3 block with the input
jobs in tx order (mixed templates per wave) versus grouped by template
(P2WPKH first, then P2PKH). Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "haskoin-node_amd"))


def main():
    import torch
    torch.cuda.init()
    import hkv
    from hkv import blockgen
    v = hkv.Verifier(hkv.VerifierConfig(device_ids=[0]))
    st = torch.cuda.Stream()
    sp = st.cuda_stream
    out = {}
    for n_tx in (2000, 64000):
        txs, inputs = blockgen.make_block(v, torch, n_tx=n_tx, seed=blockgen.SEED + n_tx)
        for label, jobs in (("tx_order", inputs), ("by_template", sorted(inputs, key=lambda j: len(j[2])))):
            db = blockgen.DeviceBlock(torch, txs, jobs)

            def extract():
                v.std_inputs_device(0, db.txs, db.d_jobs.data_ptr(), db.n, -1, db.records.data_ptr(), sp)
            extract()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(20):
                extract()
            e1.record(st)
            torch.cuda.synchronize()
            out[f"{n_tx}_{label}_us"] = round(e0.elapsed_time(e1) * 1e3 / 20, 1)
    print(json.dumps(out), flush=True)
    v.close()


if __name__ == "__main__":
    main()
