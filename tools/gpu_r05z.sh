#!/bin/bash
# Host-batch first chunk: one grid (base) vs a quarter (q4) or an eighth (q8) of a grid.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for L in base q4 q8; do
  HKV_LIB=haskoin-node_amd/lib/$L/libhkv.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu \
    -k "host_path or two_device or failover or batch_api" --timeout 200 --timeout-method thread > gpurun_out/r05z_pytest_$L.log 2>&1 \
    && echo "$L: $(tail -1 gpurun_out/r05z_pytest_$L.log)" || exit 1
done
for rep in 1 2; do
  VARIANTS="base q4 q8" BENCH_ARGS="--no-block-mix --no-config0 --no-adversarial --no-headers --no-merkle" \
    bash tools/variants.sh >> gpurun_out/r05z_variants.txt 2>&1 || exit 1
  for v in base q4 q8; do cp gpurun_out/variant_$v.log gpurun_out/variant_${v}_$rep.log; done
done
for v in base_1 q4_1 q8_1 base_2 q4_2 q8_2; do
  python3 - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/variant_{v}.log").read().strip().splitlines()[-1])
print(v, "host_path", d["host_path"]["ms"], round(d["host_path"]["verifies_per_s"] / 1e6, 1), d["host_path"]["mismatches"],
      "inproc", d["inproc"]["ms"], round(d["inproc"]["verifies_per_s"] / 1e6, 1), d["inproc"]["mismatches_vs_labels"])
PY
done
