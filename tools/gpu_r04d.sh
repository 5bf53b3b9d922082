#!/bin/bash
# Round-4 session d: the GPU suite on the in-tree build, a same-box A/B of
# library variants (tools/gpu_r04c.sh), then kernel traces of the block paths
# with the 64,000-tx batch on the in-tree build (tools/block_trace.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r04d}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_gpu.log
if [ -n "$VARIANTS" ]; then
  SKIP_BENCH=1 TAG=$TAG bash tools/gpu_r04c.sh || exit 1
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_b32 -o b32 -- \
  python3 tools/block_trace.py --k 5 --batch32 > gpurun_out/${TAG}_b32.log 2>&1 \
  && python3 tools/block_trace.py --report gpurun_out/prof_${TAG}_b32 > gpurun_out/${TAG}_b32_report.txt && echo "trace ok"
if [ -n "$FULL_BENCH" ]; then
  timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench_full.log 2>&1 && echo "full bench ok"
fi
