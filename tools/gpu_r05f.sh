#!/bin/bash
# configs[4] per-GPU rate at the shard sizes the driver's N > 1 runs use
# (16M / N records per rank), on one GPU: what the scaling line should read.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r05f}
S="--no-cpu-baseline --no-block-mix --no-config0 --no-adversarial --no-headers --no-merkle --no-host-path --no-inproc"
timeout -k 10 300 python bench.py --config4 --config4-n 2097152 --steps 10 --warmup 2 $S > gpurun_out/${TAG}_c4_2M.log 2>&1 \
  && timeout -k 10 300 python bench.py --config4 --config4-n 8388608 --steps 5 --warmup 1 $S > gpurun_out/${TAG}_c4_8M.log 2>&1 \
  && timeout -k 10 300 python bench.py --steps 10 --warmup 2 $S > gpurun_out/${TAG}_c1.log 2>&1
rc=$?
for f in gpurun_out/${TAG}_c4_2M.log gpurun_out/${TAG}_c4_8M.log gpurun_out/${TAG}_c1.log; do
  python3 - "$f" <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    print(sys.argv[1], round(d["value"] / 1e6, 2), "M/s", d["ms_per_step"], "ms/step", d["kernel_ms"], "mism", d["mismatches"],
          d["config"].get("workload", "")[:60])
except Exception as e:
    print(sys.argv[1], "unreadable", e)
PY
done
exit $rc
