#!/bin/bash
# One GPU session (round 3): the GPU suite, smoke, the default bench; each
# step under its own time limit, chained so a failure stops the session.
# TAG names the outputs under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r03}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1 \
  && echo "pytest ok" \
  && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
  && echo "smoke ok" \
  && timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.log 2>&1 \
  && echo "bench ok"
rc=$?
tail -3 gpurun_out/${TAG}_pytest_gpu.log
exit $rc
