#!/bin/bash
# Bench several libhkv builds (haskoin-node_amd/lib/<variant>/libhkv.so) in one GPU session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
rc=0
for v in ${VARIANTS}; do
  HKV_LIB=haskoin-node_amd/lib/$v/libhkv.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} \
    > gpurun_out/variant_$v.log 2>&1 || { rc=$?; echo "variant $v failed rc=$rc"; break; }
  echo "$v: $(tail -1 gpurun_out/variant_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); b=d.get("block_mix") or {}; print(d["value"], d["kernel_ms"], d["mismatches"], d["roofline"]["frac"], "config0_us", (d.get("config0") or {}).get("total_us"), "block_us", (b.get("block") or {}).get("total_us"))')"
done
exit $rc
