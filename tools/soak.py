"""Sustained throughput: the bench's 1M-record verify (BASELINE configs[1],
HKV_LIBSECP) back to back for a fixed wall time on one GPU, the rate and
the shader clock per interval — does the headline hold past the bench's
~0.2 s timed region (power / thermal)?

    python3 tools/soak.py [seconds] [interval_s] > gpurun_out/soak.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "haskoin-node_amd"))


def main(seconds: float = 120.0, interval: float = 10.0) -> None:
    import ctypes

    import numpy as np
    import torch
    import hkv
    n = 1 << 20
    v = hkv.Verifier(hkv.VerifierConfig(device_ids=[0]))
    st = torch.cuda.Stream()
    recs = torch.empty(n * 168, dtype=torch.uint8, device="cuda")
    bits = torch.zeros((n + 63) // 64 * 2, dtype=torch.int32, device="cuda")
    v.gen_records_device(0, 0x484B5632, n, 65536, 100, recs.data_ptr(), st.cuda_stream)
    st.synchronize()
    for _ in range(5):
        v.verify_device(0, recs.data_ptr(), n, 0, bits.data_ptr(), st.cuda_stream)
    st.synchronize()
    rows = []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        t0 = time.perf_counter()
        steps = 0
        while time.perf_counter() - t0 < interval:
            for _ in range(8):
                v.verify_device(0, recs.data_ptr(), n, 0, bits.data_ptr(), st.cuda_stream)
            st.synchronize()
            steps += 8
        dt = time.perf_counter() - t0
        # the clock of one more launch (profiling on for it only: its probe
        # reads the shader clock against the constant-rate counter)
        v.lib.hkv_profile_enable(v.ctx, 1)
        v.verify_device(0, recs.data_ptr(), n, 0, bits.data_ptr(), st.cuda_stream)
        st.synchronize()
        sclk = ctypes.c_double()
        v.lib.hkv_profile_clock(v.ctx, 0, ctypes.byref(sclk))
        v.lib.hkv_profile_enable(v.ctx, 0)
        rows.append({"t_s": round(time.perf_counter() - (t_end - seconds), 1), "verifies_per_s": round(n * steps / dt, 1),
                     "steps": steps, "sclk_mhz": round(sclk.value, 1) if 500 < sclk.value < 4000 else None})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    got = bits.cpu().numpy().view(np.uint32)
    accepted = int(np.unpackbits(got.view(np.uint8), bitorder="little")[:n].sum())
    rates = [r["verifies_per_s"] for r in rows]
    print(json.dumps({"workload": "BASELINE configs[1]: 1,048,576 valid records, HBM-resident, back to back",
                      "seconds": seconds, "intervals": rows, "accepted_last": accepted,
                      "rate_first": rates[0], "rate_last": rates[-1], "rate_min": min(rates),
                      "rate_median": sorted(rates)[len(rates) // 2]}))
    v.close()


if __name__ == "__main__":
    main(float(sys.argv[1]) if len(sys.argv) > 1 else 120.0, float(sys.argv[2]) if len(sys.argv) > 2 else 10.0)
