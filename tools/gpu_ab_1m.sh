#!/bin/bash
# Same-box A/B of the 1M headline (BASELINE configs[1]) between the in-tree
# build and a baseline library (haskoin-node_amd/lib/libhkv_base.so, HKV_LIB),
# two alternations, then the FETCH_SIZE / WRITE_SIZE passes of the ecmult
# launch for both builds (one counter group per run, as MI355X_MICROARCH.md
# prescribes). TAG names the outputs under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-ab1m}
BASE=haskoin-node_amd/lib/libhkv_base.so
B="bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-block-mix --no-config0 --no-adversarial --no-headers --no-merkle --no-host-path --no-inproc"
for k in 1 2; do
  HKV_LIB=$BASE timeout -k 10 200 python $B > gpurun_out/${TAG}_base$k.log 2>&1 || exit 1
  timeout -k 10 200 python $B > gpurun_out/${TAG}_new$k.log 2>&1 || exit 1
done
P="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-block-mix --no-config0 --no-adversarial --no-headers --no-merkle --no-host-path --no-inproc"
for v in base new; do
  for c in FETCH_SIZE WRITE_SIZE; do
    if [ $v = base ]; then export HKV_LIB=$BASE; else unset HKV_LIB; fi
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_pmc_${v}_$c -o p -- python3 $P \
      > gpurun_out/${TAG}_pmc_${v}_$c.log 2>&1 || exit 1
  done
done
unset HKV_LIB
for f in gpurun_out/${TAG}_base1.log gpurun_out/${TAG}_new1.log gpurun_out/${TAG}_base2.log gpurun_out/${TAG}_new2.log; do
  python3 - "$f" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "value", round(d["value"] / 1e6, 2), "ecmult_ms", d["kernel_ms"]["ecmult"], "frac", d["roofline"]["frac"],
      "sclk", d["roofline"].get("sclk_mhz"), "mismatches", d["mismatches"])
PY
done
python3 tools/pmc_kernel_bytes.py gpurun_out/${TAG}_pmc_base_FETCH_SIZE gpurun_out/${TAG}_pmc_base_WRITE_SIZE \
  gpurun_out/${TAG}_pmc_new_FETCH_SIZE gpurun_out/${TAG}_pmc_new_WRITE_SIZE > gpurun_out/${TAG}_pmc_summary.txt 2>&1
tail -20 gpurun_out/${TAG}_pmc_summary.txt
