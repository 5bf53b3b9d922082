"""Block files for tools/native_latency.cpp and tools/native_concurrency.cpp:
BASELINE configs[0] (or the configs[2] block mix, or a 600-tx multisig block)
as the tx bytes, the n_tx + 1 offsets, the script pool and the hkv_input_job
array, in the layouts include/hkv.h defines.

    python3 tools/native_latency.py dump gpurun_out/blk0 [config0|config2|multisig]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "haskoin-node_amd"))


def dump(out_dir: str, which: str = "config0") -> None:
    import numpy as np
    import torch
    import hkv
    from hkv import blockgen
    from hkv.sighash import INPUT_JOB_DTYPE, TxBatch
    os.makedirs(out_dir, exist_ok=True)
    with hkv.Verifier(hkv.VerifierConfig(device_ids=[0], flags=1)) as v:
        if which == "config0":
            txs, inputs = blockgen.make_p2pkh_block(v, torch)
        elif which == "multisig":
            txs, inputs = blockgen.make_multisig_block(v, torch, n_tx=600)
        else:
            txs, inputs = blockgen.make_block(v, torch)
    tb = TxBatch(txs)
    jobs = np.zeros(len(inputs), dtype=INPUT_JOB_DTYPE)
    for k, (t, i, spk, value) in enumerate(inputs):
        off, ln = tb.script(spk)
        jobs[k] = (t, i, off, ln, value)
    _, pool = tb.struct()
    for name, arr in (("txs", tb.bytes), ("offsets", tb.offsets), ("scripts", pool), ("jobs", jobs)):
        np.ascontiguousarray(arr).tofile(os.path.join(out_dir, name + ".bin"))
    print(f"{which}: {len(txs)} txs, {len(inputs)} inputs -> {out_dir}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) < 3 or sys.argv[1] != "dump":
        sys.exit(__doc__)
    dump(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "config0")
