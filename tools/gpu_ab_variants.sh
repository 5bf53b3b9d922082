#!/bin/bash
# Same-box A/B of library variants (compiler-flag builds of the same source):
# the 1M headline and the configs[0] / configs[2] block legs, alternated.
#   VARIANTS="maxilp memclause" TAG=r06r bash tools/gpu_ab_variants.sh
# (haskoin-node_amd/lib/libhkv_<v>.so; "base" = the in-tree libhkv.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-abvar}
B="bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-adversarial --no-headers --no-merkle --no-host-path --no-inproc --no-checker"
for k in 1 2; do
  for v in base ${VARIANTS}; do
    if [ $v = base ]; then unset HKV_LIB; else export HKV_LIB=haskoin-node_amd/lib/libhkv_$v.so; fi
    timeout -k 10 300 python $B > gpurun_out/${TAG}_${v}_$k.log 2>&1 || exit 1
  done
done
unset HKV_LIB
for f in gpurun_out/${TAG}_*_[12].log; do
  python3 - "$f" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
m = d.get("block_mix") or {}
print(sys.argv[1], "value", round(d["value"] / 1e6, 2), "ecmult_ms", d["kernel_ms"]["ecmult"], "sclk",
      d["roofline"].get("sclk_mhz"), "mism", d["mismatches"], "c0_us", (d.get("config0") or {}).get("total_us"),
      "c2_us", (m.get("block") or {}).get("total_us"), "pool16k_us", (m.get("pool16k") or {}).get("total_us"))
PY
done
