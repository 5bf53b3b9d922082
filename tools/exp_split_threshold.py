"""Experiment: ecmult launch time vs batch size, to place the split-lane
threshold (run once per libhkv build: HKV_LIB=... python tools/exp_split_threshold.py)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "haskoin-node_amd"))


def main():
    import torch
    torch.cuda.init()
    import hkv
    v = hkv.Verifier(hkv.VerifierConfig(device_ids=[0]))
    st = torch.cuda.Stream()
    sp = st.cuda_stream
    out = {}
    for n in (8192, 16384, 24576, 32768, 49152, 65536, 98304, 131072):
        recs = torch.empty(n * 168, dtype=torch.uint8, device="cuda")
        bits = torch.zeros((n + 63) // 64 * 2, dtype=torch.int32, device="cuda")
        v.gen_records_device(0, 77 + n, n, 65536, 100, recs.data_ptr(), sp)
        v.verify_device(0, recs.data_ptr(), n, 0, bits.data_ptr(), sp)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(10):
            v.verify_device(0, recs.data_ptr(), n, 0, bits.data_ptr(), sp)
        e1.record(st)
        torch.cuda.synchronize()
        acc = int(bits.cpu().numpy().view("uint32").astype("uint64").tolist().__len__())
        out[str(n)] = round(e0.elapsed_time(e1) * 1e3 / 10, 1)
    print(json.dumps({"lib": os.environ.get("HKV_LIB", "default"), "verify_us": out}), flush=True)
    v.close()


if __name__ == "__main__":
    main()
