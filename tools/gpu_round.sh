#!/bin/bash
# One GPU session: parity tests, smoke, bench. Each GPU step has its own
# time limit; steps are chained so a failure stops the session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -m pytest tests -x -q -m gpu ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 \
  && echo "pytest ok" \
  && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
  && echo "smoke ok" \
  && timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 \
  && echo "bench ok"
rc=$?
tail -5 gpurun_out/pytest_gpu.log
tail -3 gpurun_out/bench.log 2>/dev/null
exit $rc
