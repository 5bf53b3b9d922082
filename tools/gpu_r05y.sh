#!/bin/bash
# Host-batch chunk schedule (geometric, first chunk one grid): the GPU suite
# on the in-tree build, then base / geo benches of the PCIe-inclusive legs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05y_pytest.log 2>&1 \
  && tail -1 gpurun_out/r05y_pytest.log || exit 1
VARIANTS="base geo base geo" BENCH_ARGS="--no-block-mix --no-config0 --no-adversarial --no-headers --no-merkle" \
  bash tools/variants.sh || exit 1
for v in base geo; do
  python3 - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/variant_{v}.log").read().strip().splitlines()[-1])
print(v, "host_path", d["host_path"]["ms"], round(d["host_path"]["verifies_per_s"] / 1e6, 1), d["host_path"]["mismatches"],
      "inproc", d["inproc"]["ms"], round(d["inproc"]["verifies_per_s"] / 1e6, 1), d["inproc"]["mismatches_vs_labels"])
PY
done
