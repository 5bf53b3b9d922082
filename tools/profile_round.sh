#!/bin/bash
# rocprofv3 evidence for the bench kernels: kernel trace + stats, then PMC
# passes (one counter group per run; no sys/runtime trace with --pmc).
# Usage (on the GPU box): tools/profile_round.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r01}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
# trace pass: the whole default bench (every section); PMC passes: the 1M
# verify only, so the ecmult counters are those of the timed launch
# (--no-host-path / --no-inproc: their hkv_verify chunks run the same 262,144-lane
# ecmult grid over more records per launch and would mix into its statistics)
FULL="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-host-path --no-inproc ${BENCH_ARGS}"
BENCH="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-block-mix --no-config0 --no-adversarial --no-headers --no-merkle --no-host-path --no-inproc ${BENCH_ARGS}"
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o "$name" -- python3 $BENCH \
    > "$OUT/$name.log" 2>&1
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- python3 $FULL \
    > "$OUT/trace.log" 2>&1 \
 && run pmc_valu --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
 && run pmc_busy --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
 && run pmc_occ --pmc SQ_LEVEL_WAVES SQ_ACCUM_PREV_HIRES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
 && run pmc_fetch --pmc FETCH_SIZE \
 && run pmc_write --pmc WRITE_SIZE
rc=$?
ls -R "$OUT" | head -50
exit $rc
