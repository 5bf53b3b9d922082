#!/bin/bash
# The final build's node-view numbers: the isolated tip-block call under a
# rocprofv3 kernel trace (tools/isolated_call.py), configs[4] at the N > 1
# shard sizes (tools/gpu_r05f.sh), and a 120-s sustained 1M run (soak.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=r05t2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_${TAG}_iso -o iso \
    -- python3 tools/isolated_call.py run gpurun_out/${TAG}_iso_host.json > gpurun_out/${TAG}_iso.log 2>&1 \
  && python3 tools/isolated_call.py report gpurun_out/prof_${TAG}_iso gpurun_out/${TAG}_iso_host.json \
       > gpurun_out/${TAG}_iso_report.json 2>&1 && echo "iso ok" && cat gpurun_out/${TAG}_iso_report.json \
  && TAG=${TAG} timeout -k 10 600 bash tools/gpu_r05f.sh \
  && timeout -k 10 200 python3 tools/soak.py 120 15 > gpurun_out/${TAG}_soak.json 2> gpurun_out/${TAG}_soak.err \
  && echo "soak ok" && cat gpurun_out/${TAG}_soak.json
