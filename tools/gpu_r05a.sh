#!/bin/bash
# Round-5 session A: the new GPU tests first (multisig tail: stale rows,
# barrier fault reporting; malformed wire data on the block kernel; the
# share-device spawn), then the whole GPU suite, smoke, the default bench
# (steady-state CPU baseline), and a same-box A/B of the cooperative tail
# launch against a plain one (libhkv_nocoop.so, HKV_LIB) on the block legs.
# Each GPU step has its own time limit; steps are chained.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r05a}
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT -m gpu tests/test_gpu_sighash.py -k "tail or malformed" tests/test_gpu_spawn.py \
    > gpurun_out/${TAG}_pytest_new.log 2>&1 \
  && echo "new tests ok" \
  && timeout -k 10 900 $PT -m gpu tests > gpurun_out/${TAG}_pytest_gpu.log 2>&1 \
  && echo "pytest ok" \
  && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
  && echo "smoke ok" \
  && timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 \
  && echo "bench ok" || { rc=$?; tail -30 gpurun_out/${TAG}_pytest_new.log; tail -5 gpurun_out/${TAG}_pytest_gpu.log; exit $rc; }
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-adversarial --no-headers --no-merkle --no-host-path --no-inproc"
for k in 1 2; do
  HKV_LIB=haskoin-node_amd/lib/libhkv_nocoop.so timeout -k 10 200 python $B > gpurun_out/${TAG}_plain$k.log 2>&1 || exit 1
  timeout -k 10 200 python $B > gpurun_out/${TAG}_coop$k.log 2>&1 || exit 1
done
for f in gpurun_out/${TAG}_plain1.log gpurun_out/${TAG}_coop1.log gpurun_out/${TAG}_plain2.log gpurun_out/${TAG}_coop2.log; do
  python3 - "$f" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b = d["block_mix"]
print(sys.argv[1], "config0_us", d["config0"]["total_us"], "lat", d["config0"]["latency_us"], "block_us",
      b["block"]["total_us"], "pool16k_us", b["pool16k"]["total_us"], "batch32_us", b["batch32"]["total_us"],
      "value", round(d["value"] / 1e6, 2), "sclk", d["roofline"].get("sclk_mhz"))
PY
done
tail -3 gpurun_out/${TAG}_pytest_gpu.log
