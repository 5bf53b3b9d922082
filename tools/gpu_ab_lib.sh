#!/bin/bash
# Same-box A/B of the in-tree build against a baseline library
# (haskoin-node_amd/lib/libhkv_base.so, HKV_LIB): the GPU suite on the
# in-tree build, then the bench's block sections alternating base / new.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-ablib}
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-adversarial --no-headers --no-merkle --no-host-path"
timeout -k 10 ${PYTEST_LIMIT:-900} python -u -m pytest tests -x -v -m gpu --timeout 800 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 \
  && echo "pytest ok" && tail -1 gpurun_out/${TAG}_pytest.log || exit 1
for k in 1 2; do
  HKV_LIB=haskoin-node_amd/lib/libhkv_base.so timeout -k 10 200 python $B > gpurun_out/${TAG}_base$k.log 2>&1 || exit 1
  timeout -k 10 200 python $B > gpurun_out/${TAG}_new$k.log 2>&1 || exit 1
done
for f in gpurun_out/${TAG}_base1.log gpurun_out/${TAG}_new1.log gpurun_out/${TAG}_base2.log gpurun_out/${TAG}_new2.log; do
  python3 - "$f" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b = d["block_mix"]
print(sys.argv[1], "config0_us", d["config0"]["total_us"], "block_us", b["block"]["total_us"],
      "pool16k_us", b["pool16k"]["total_us"], "batch32_us", b["batch32"]["total_us"], "value", round(d["value"] / 1e6, 2), "sclk", d["roofline"].get("sclk_mhz"))
PY
done
