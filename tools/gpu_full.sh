#!/bin/bash
# Full GPU session: parity tests, smoke, bench (N=1), torchrun N=1 bench
# (exercises the RCCL path), rocprofv3 trace + PMC passes. Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r01}
./tools/gpu_round.sh \
  && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
       --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_torchrun.log 2>&1 \
  && echo "torchrun ok" \
  && ./tools/profile_round.sh "$TAG" > gpurun_out/profile_${TAG}.log 2>&1 \
  && echo "profile ok"
