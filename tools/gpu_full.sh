#!/bin/bash
# Full GPU session: parity tests, smoke, bench (N=1), a torchrun N=1 bench with
# --force-collective (a one-rank nccl/RCCL group with device_id and the step's
# device-side all-gather; without the flag a world-1 run creates no group and
# runs no collective), rocprofv3 trace + PMC passes. Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r01}
./tools/gpu_round.sh \
  && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
       --master-port 29533 bench.py --gpus 1 --force-collective --config4 --steps 5 --warmup 1 > gpurun_out/bench_torchrun.log 2>&1 \
  && echo "torchrun ok" \
  && ./tools/profile_round.sh "$TAG" > gpurun_out/profile_${TAG}.log 2>&1 \
  && echo "profile ok"
