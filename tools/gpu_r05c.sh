#!/bin/bash
# Round-5 session C: the GPU suite on the build that skips the scratch wait
# on the last stream; the isolated tip-block call (rocprofv3 kernel trace of
# tools/isolated_call.py) for the new build and for libhkv_base.so; the bench
# block legs A/B (base = round-5 build before the skip).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r05c}
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT -m gpu tests > gpurun_out/${TAG}_pytest_gpu.log 2>&1 && echo "pytest ok" \
  || { rc=$?; grep -v PASSED gpurun_out/${TAG}_pytest_gpu.log | tail -30; exit $rc; }
for lib in new base; do
  if [ $lib = base ]; then export HKV_LIB=haskoin-node_amd/lib/libhkv_base.so; else unset HKV_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_${TAG}_iso_$lib -o iso \
      -- python3 tools/isolated_call.py run gpurun_out/${TAG}_iso_host_$lib.json > gpurun_out/${TAG}_iso_$lib.log 2>&1 \
    && python3 tools/isolated_call.py report gpurun_out/prof_${TAG}_iso_$lib gpurun_out/${TAG}_iso_host_$lib.json \
         > gpurun_out/${TAG}_iso_report_$lib.json 2>&1 || exit 1
  echo "== $lib"; cat gpurun_out/${TAG}_iso_report_$lib.json
done
unset HKV_LIB
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-adversarial --no-headers --no-merkle --no-host-path --no-inproc"
for k in 1 2; do
  HKV_LIB=haskoin-node_amd/lib/libhkv_base.so timeout -k 10 200 python $B > gpurun_out/${TAG}_base$k.log 2>&1 || exit 1
  timeout -k 10 200 python $B > gpurun_out/${TAG}_new$k.log 2>&1 || exit 1
done
for f in gpurun_out/${TAG}_{base,new}{1,2}.log; do
  python3 - "$f" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b = d["block_mix"]
print(sys.argv[1].split("/")[-1], "config0_us", d["config0"]["total_us"], "latency_us", d["config0"]["latency_us"],
      "block_us", b["block"]["total_us"], "latency_block", b["block"]["latency_us"], "pool16k_us", b["pool16k"]["total_us"],
      "batch32_us", b["batch32"]["total_us"], "value", round(d["value"] / 1e6, 2), "sclk", d["roofline"].get("sclk_mhz"))
PY
done
