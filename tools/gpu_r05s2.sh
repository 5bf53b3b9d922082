#!/bin/bash
# The opt-in stress tests on the final build (after the top-window merge):
# record byte mutations, wire mutations through the block kernel, seeded
# multisig blocks, overlapping callers. Outputs under gpurun_out/r05s2_*.log.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
P="python -u -m pytest -s -x -v -m gpu --timeout 900 --timeout-method thread"
HKV_STRESS_RECORD_BATCHES=60 timeout -k 10 400 $P tests/test_gpu_parity.py -k record_byte_mutation_stress \
    > gpurun_out/r05s2_records.log 2>&1 && echo "records ok" \
 && HKV_STRESS_SEEDS=300 timeout -k 10 400 $P tests/test_gpu_sighash.py -k wire_mutation_stress \
    > gpurun_out/r05s2_wire.log 2>&1 && echo "wire ok" \
 && HKV_STRESS_MS_BLOCKS=36 timeout -k 10 400 $P tests/test_gpu_sighash.py -k multisig_block_stress \
    > gpurun_out/r05s2_multisig.log 2>&1 && echo "multisig ok" \
 && HKV_STRESS_ROUNDS=400 timeout -k 10 200 $P tests/test_gpu_concurrency.py \
    > gpurun_out/r05s2_concurrency.log 2>&1 && echo "concurrency ok"
