#!/bin/bash
# The tip block from a native caller (tools/native_latency.cpp): configs[0]
# and the configs[2] block mix, each timed back to back, alone, and alone
# after 5 ms of GPU idle.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r05h}
timeout -k 10 200 python3 tools/native_latency.py dump gpurun_out/blk0 config0 \
  && timeout -k 10 200 python3 tools/native_latency.py dump gpurun_out/blk2 config2 \
  && timeout -k 10 120 tools/native_latency gpurun_out/blk0 > gpurun_out/${TAG}_native_config0.json \
  && timeout -k 10 120 tools/native_latency gpurun_out/blk2 > gpurun_out/${TAG}_native_config2.json \
  && cat gpurun_out/${TAG}_native_config0.json gpurun_out/${TAG}_native_config2.json
