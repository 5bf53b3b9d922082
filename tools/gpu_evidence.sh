#!/bin/bash
# One evidence session on the committed build: the GPU suite, smoke, the
# default bench (every section, CPU baseline included), the rocprofv3 kernel
# trace + PMC passes of tools/profile_round.sh, and the block-path kernel
# trace with the 64,000-tx batch (tools/block_trace.py --batch32). TAG names the outputs under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r04}
export TMPDIR=/tmp
TAG=$TAG bash tools/gpu_r04.sh \
  && bash tools/profile_round.sh $TAG \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_block -o block \
       -- python3 tools/block_trace.py --batch32 > gpurun_out/${TAG}_block_trace.log 2>&1 \
  && python3 tools/block_trace.py --report gpurun_out/prof_${TAG}_block > gpurun_out/${TAG}_block_report.log 2>&1 \
  && echo "evidence ok"
