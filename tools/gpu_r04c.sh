#!/bin/bash
# Round-4 session: same-box A/B of library variants (haskoin-node_amd/lib/<v>/libhkv.so,
# two alternations), the default bench on the in-tree build (with the in-process
# all-GPU leg), and a PMC pass over the block paths (tools/block_trace.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r04c}
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-adversarial --no-host-path --no-inproc --no-headers --no-merkle"
for k in 1 2; do
  for v in ${VARIANTS}; do
    HKV_LIB=haskoin-node_amd/lib/$v/libhkv.so timeout -k 10 240 python $B > gpurun_out/${TAG}_${v}_$k.log 2>&1 \
      || { echo "variant $v failed"; exit 1; }
    python3 - gpurun_out/${TAG}_${v}_$k.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
b = d["block_mix"]
print(sys.argv[1], "value", round(d["value"] / 1e6, 2), "ecm_ms", d["kernel_ms"]["ecmult"], "config0", d["config0"]["total_us"],
      d["config0"].get("latency_us"), "block", b["block"]["total_us"], b["block"].get("latency_us"), "batch32",
      b["batch32"]["total_us"], "sclk", d["roofline"].get("sclk_mhz"))
PY
  done
done
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 && echo "bench ok" \
  && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_INT64 \
       --output-format csv -d gpurun_out/prof_${TAG}_blockpmc -o pmc -- python3 tools/block_trace.py --k 3 > gpurun_out/${TAG}_blockpmc.log 2>&1 \
  && echo "pmc ok"
