#!/bin/bash
# PMC pass for instruction-fetch / I-cache behaviour of the bench kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-icache}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC \
  --output-format csv -d "$OUT/ic" -o ic -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/ic.log" 2>&1
