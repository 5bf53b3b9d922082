#!/bin/bash
# Print the small-batch latencies (configs[2] block, 32-block batch) of the variant logs tools/variants.sh wrote.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in ${VARIANTS}; do
  python3 - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/variant_{v}.log").read().strip().splitlines()[-1])
b = d["block_mix"]
print(v, b["block"]["total_us"], b["block"]["extract_sighash_us"], b["batch32"]["total_us"], b["batch32"].get("extract_sighash_us"))
PY
done
