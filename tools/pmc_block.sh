#!/bin/bash
# PMC passes over the block kernel (configs[0] and configs[2] legs of the
# bench): VALU issue / busy and instruction mix per dispatch, so the block
# kernel's bound (one wave per SIMD, issue-limited) is measured, not assumed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-blk}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-adversarial --no-headers --no-merkle --no-host-path --no-inproc"
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/busy" -o busy -- python3 $B > "$OUT/busy.log" 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
  --output-format csv -d "$OUT/valu" -o valu -- python3 $B > "$OUT/valu.log" 2>&1
