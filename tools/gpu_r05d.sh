#!/bin/bash
# Round-5 evidence session: the GPU suite, smoke, the default bench twice on
# one box (cpu_baseline steady-state agreement), the --share-device spawn
# leg, then tools/profile_round.sh (kernel trace + PMC passes). TAG names
# the outputs under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r05d}
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1 && echo "pytest ok" \
  && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
  && echo "smoke ok" \
  && timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench1.log 2>&1 && echo "bench1 ok" \
  && timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench2.log 2>&1 && echo "bench2 ok" \
  && timeout -k 10 300 python bench.py --gpus 2 --share-device --config4-n 2097152 --steps 5 --warmup 1 \
       > gpurun_out/${TAG}_spawn2.log 2>&1 && echo "spawn2 ok" \
  && timeout -k 10 120 python bench.py --gpus 2 --steps 2 > gpurun_out/${TAG}_gpus2.log 2>&1; rc=$?
echo "--gpus 2 on the 1-GPU lease: rc=$rc (want 2)"
[ $rc -eq 2 ] || { grep -v PASSED gpurun_out/${TAG}_pytest_gpu.log | tail -20; exit 1; }
bash tools/profile_round.sh $TAG && echo "profile ok"
