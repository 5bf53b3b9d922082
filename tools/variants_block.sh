#!/bin/bash
# Print the small-batch latencies (configs[0] and configs[2] blocks, 32-block batch) and the headline of the variant logs tools/variants.sh wrote.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in ${VARIANTS}; do
  python3 - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/variant_{v}.log").read().strip().splitlines()[-1])
b = d["block_mix"]
print(v, "config0_us", d.get("config0", {}).get("total_us"), "block_us", b["block"]["total_us"],
      "batch32_us", b["batch32"]["total_us"], "value", d["value"])
PY
done
