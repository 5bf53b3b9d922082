#!/bin/bash
# One GPU session for a kernel change: field microbenchmark (with its
# new-vs-reference check), the GPU parity suite on the default build, then a
# same-box A/B of variant builds (tools/variants.sh). Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${TAG:-ab}
timeout -k 10 180 ./tools/ubench_field > gpurun_out/ubench_${TAG}.json 2>&1 \
  && echo "ubench ok" && head -1 gpurun_out/ubench_${TAG}.json \
  && timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1 \
  && echo "pytest ok" && tail -1 gpurun_out/pytest_${TAG}.log \
  && ./tools/variants.sh
rc=$?
tail -3 gpurun_out/pytest_${TAG}.log 2>/dev/null
exit $rc
