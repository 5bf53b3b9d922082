#!/bin/bash
# One GPU session (round 4): the launcher's fail-fast check (--gpus 2 on a
# 1-GPU lease must exit 2 before starting ranks), the GPU suite, smoke, the
# bench, the bench under torchrun at N = 1; each step under its own time limit, chained so a failure stops the
# session. TAG names the outputs under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r04}
timeout -k 10 120 python bench.py --gpus 2 --steps 2 > gpurun_out/${TAG}_gpus2.log 2>&1
rc=$?
echo "bench --gpus 2 on one GPU: rc=$rc (want 2)"; tail -2 gpurun_out/${TAG}_gpus2.log
[ $rc -eq 2 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1 \
  && echo "pytest ok" \
  && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
  && echo "smoke ok" \
  && timeout -k 10 600 python bench.py --gpus 1 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.log 2>&1 \
  && echo "bench ok" \
  && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
       --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu-baseline --no-block-mix --no-config0 \
       --no-adversarial --no-headers --no-merkle --no-host-path --no-inproc > gpurun_out/${TAG}_bench_torchrun.log 2>&1 \
  && echo "torchrun bench ok"
rc=$?
tail -3 gpurun_out/${TAG}_pytest_gpu.log
exit $rc
