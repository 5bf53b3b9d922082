#!/bin/bash
# Round-5 session B: the lane-split product prototype (tools/ubench_chain:
# correctness check, then lone-wave cycles), the multisig tail as an ordered
# work queue (its GPU tests first, then the whole suite), and a same-box A/B
# of the block legs against the grid-barrier tail (libhkv_base.so, HKV_LIB)
# and the lane-split quad doubling (libhkv_qsplit.so, -DHKV_QUAD_SPLIT=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r05b}
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 120 ./tools/ubench_chain > gpurun_out/${TAG}_ubench_chain.json 2>&1; echo "ubench rc=$?"; cat gpurun_out/${TAG}_ubench_chain.json
timeout -k 10 600 $PT -m gpu tests/test_gpu_sighash.py -k "tail or multisig or malformed" > gpurun_out/${TAG}_pytest_new.log 2>&1 \
  && echo "tail tests ok" \
  && timeout -k 10 900 $PT -m gpu tests > gpurun_out/${TAG}_pytest_gpu.log 2>&1 \
  && echo "pytest ok" || { rc=$?; grep -v PASSED gpurun_out/${TAG}_pytest_new.log | tail -30; tail -5 gpurun_out/${TAG}_pytest_gpu.log; exit $rc; }
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-adversarial --no-headers --no-merkle --no-host-path --no-inproc"
for k in 1 2; do
  HKV_LIB=haskoin-node_amd/lib/libhkv_base.so timeout -k 10 200 python $B > gpurun_out/${TAG}_base$k.log 2>&1 || exit 1
  timeout -k 10 200 python $B > gpurun_out/${TAG}_new$k.log 2>&1 || exit 1
  HKV_LIB=haskoin-node_amd/lib/libhkv_qsplit.so timeout -k 10 200 python $B > gpurun_out/${TAG}_qsplit$k.log 2>&1 || exit 1
done
for f in gpurun_out/${TAG}_{base,new,qsplit}{1,2}.log; do
  python3 - "$f" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b = d["block_mix"]
print(sys.argv[1].split("/")[-1], "config0_us", d["config0"]["total_us"], "latency_us", d["config0"]["latency_us"],
      "block_us", b["block"]["total_us"], "pool16k_us", b["pool16k"]["total_us"], "batch32_us", b["batch32"]["total_us"],
      "value", round(d["value"] / 1e6, 2), "sclk", d["roofline"].get("sclk_mhz"))
PY
done
tail -2 gpurun_out/${TAG}_pytest_gpu.log
