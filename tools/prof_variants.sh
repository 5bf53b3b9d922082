#!/bin/bash
# Kernel-trace stats of one bench run per variant build
# (haskoin-node_amd/lib/<variant>/libhkv.so), for per-kernel A/B durations.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rc=0
for v in ${VARIANTS}; do
  HKV_LIB=haskoin-node_amd/lib/$v/libhkv.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$v -o run \
    -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$v.log 2>&1 || { rc=$?; echo "variant $v failed rc=$rc"; break; }
  echo "$v done"
done
exit $rc
