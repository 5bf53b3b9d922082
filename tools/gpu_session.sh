#!/bin/bash
# GPU sessions on the committed build (one gpurun call each); outputs under
# gpurun_out/<TAG>_*. Every GPU step runs under its own time limit and the
# steps are chained, so the first failure ends the session.
#
#   tools/gpu_session.sh suite TAG     the GPU suite and smoke (evidence's first half)
#   tools/gpu_session.sh benches TAG   evidence's second half (from the benches on);
#                                      the two halves fit gpurun's 1,200-s limit
#                                      where the whole session may not
#   tools/gpu_session.sh evidence TAG  the GPU suite, smoke, the default bench
#                                      twice (cpu_baseline agreement), the
#                                      --share-device two-rank spawn, the
#                                      one-rank RCCL all-gather (--force-collective,
#                                      spawned and under torchrun),
#                                      --gpus 2 fail-fast on a 1-GPU lease, then
#                                      tools/profile_round.sh (kernel trace + PMC)
#   tools/gpu_session.sh node TAG      the node's view: the isolated tip-block
#                                      call under a kernel trace, the native C ABI
#                                      caller, configs[4] at the N > 1 shard sizes,
#                                      an IBD-sized verifyStdInput batch (--std-ibd),
#                                      a 120-s sustained 1M run
#   tools/gpu_session.sh stress TAG    the opt-in stress tests (record / wire
#                                      mutations, multisig blocks — also with the
#                                      tail's record windows forced small —,
#                                      overlapping callers)
#
# Same-box A/Bs against haskoin-node_amd/lib/libhkv_base.so: tools/gpu_ab_lib.sh
# (block legs) and tools/gpu_ab_1m.sh (the 1M headline + traffic).
# (This script replaces the per-session tools/gpu_r0*.sh scripts of rounds
# 3-5; profiles/README_r05.md names them, git history keeps them.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
MODE=${1:?mode: evidence | suite | benches | node | stress}
TAG=${2:-$MODE}
O=gpurun_out/${TAG}
S="--no-cpu-baseline --no-block-mix --no-config0 --no-adversarial --no-headers --no-merkle --no-host-path --no-inproc"

summary() {  # bench JSON lines -> one line each
  for f in "$@"; do
    python3 - "$f" <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    c0 = (d.get("config0") or {}).get("total_us")
    print(sys.argv[1], round(d["value"] / 1e6, 2), "M/s", d["ms_per_step"], "ms/step", "frac",
          d["roofline"]["frac"], "mism", d["mismatches"], "vs_checker", (d.get("mismatches_vs_checker") or {}).get("mismatches"),
          "config0_us", c0, "collective", d.get("collective"))
except Exception as e:
    print(sys.argv[1], "unreadable", e)
PY
  done
}

suite_half() {
  timeout -k 10 1100 python -u -m pytest -x -v -m gpu --timeout 800 --timeout-method thread tests \
      > ${O}_pytest_gpu.log 2>&1 && echo "pytest ok" && tail -1 ${O}_pytest_gpu.log \
    && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1 && echo "smoke ok"
}

benches_half() {
  timeout -k 10 600 python bench.py > ${O}_bench1.log 2>&1 && echo "bench1 ok" \
    && timeout -k 10 600 python bench.py > ${O}_bench2.log 2>&1 && echo "bench2 ok" \
    && timeout -k 10 300 python bench.py --gpus 2 --share-device --config4-n 2097152 --steps 5 --warmup 1 \
         > ${O}_spawn2.log 2>&1 && echo "spawn2 ok" \
    && timeout -k 10 300 python bench.py --gpus 1 --force-collective --config4 --steps 5 --warmup 1 \
         > ${O}_rccl1.log 2>&1 && echo "rccl1 ok" \
    && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
         --master-port 29533 bench.py --gpus 1 --force-collective --config4 --steps 5 --warmup 1 \
         > ${O}_torchrun_rccl1.log 2>&1 && echo "torchrun rccl1 ok" \
    && { timeout -k 10 120 python bench.py --gpus 2 --steps 2 > ${O}_gpus2.log 2>&1; rc=$?;
         echo "--gpus 2 on the 1-GPU lease: rc=$rc (want 2)"; [ $rc -eq 2 ]; } \
    && summary ${O}_bench1.log ${O}_bench2.log ${O}_rccl1.log ${O}_torchrun_rccl1.log \
    && bash tools/profile_round.sh $TAG && echo "profile ok"
}

case "$MODE" in
evidence)
  suite_half && benches_half
  ;;
suite)
  suite_half
  ;;
benches)
  benches_half
  ;;
node)
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_${TAG}_iso -o iso \
      -- python3 tools/isolated_call.py run ${O}_iso_host.json > ${O}_iso.log 2>&1 \
    && python3 tools/isolated_call.py report gpurun_out/prof_${TAG}_iso ${O}_iso_host.json > ${O}_iso_report.json 2>&1 \
    && echo "iso ok" && cat ${O}_iso_report.json \
    && timeout -k 10 200 python3 tools/native_latency.py dump gpurun_out/blk0 config0 \
    && timeout -k 10 200 python3 tools/native_latency.py dump gpurun_out/blk2 config2 \
    && timeout -k 10 120 tools/native_latency gpurun_out/blk0 > ${O}_native_config0.json \
    && timeout -k 10 120 tools/native_latency gpurun_out/blk2 > ${O}_native_config2.json \
    && timeout -k 10 300 python bench.py --config4 --config4-n 2097152 --steps 10 --warmup 2 $S > ${O}_c4_2M.log 2>&1 \
    && timeout -k 10 300 python bench.py --config4 --config4-n 8388608 --steps 5 --warmup 1 $S > ${O}_c4_8M.log 2>&1 \
    && timeout -k 10 300 python bench.py --steps 10 --warmup 2 $S > ${O}_c1.log 2>&1 \
    && timeout -k 10 400 python bench.py --steps 8 --warmup 1 --std-ibd 560000 --no-cpu-baseline --no-config0 \
         --no-adversarial --no-headers --no-merkle --no-host-path --no-inproc --no-checker > ${O}_ibd.log 2>&1 \
    && summary ${O}_c4_2M.log ${O}_c4_8M.log ${O}_c1.log \
    && timeout -k 10 200 python3 tools/soak.py 120 15 > ${O}_soak.json 2> ${O}_soak.err \
    && echo "soak ok" && cat ${O}_soak.json
  ;;
stress)
  # STRESS_X scales every count and time limit (1: ~15 min; the records
  # stress also checks OpenSSL when HKV_STRESS_OPENSSL=1)
  X=${STRESS_X:-1}
  P="python -u -m pytest -s -x -v -m gpu --timeout $((900 * X)) --timeout-method thread"
  HKV_STRESS_RECORD_BATCHES=$((60 * X)) timeout -k 10 $((400 * X)) $P tests/test_gpu_parity.py \
      -k record_byte_mutation_stress > ${O}_records.log 2>&1 && echo "records ok" \
    && HKV_STRESS_SEEDS=$((300 * X)) timeout -k 10 $((400 * X)) $P tests/test_gpu_sighash.py -k wire_mutation_stress \
      > ${O}_wire.log 2>&1 && echo "wire ok" \
    && HKV_STRESS_MS_BLOCKS=$((36 * X)) timeout -k 10 $((400 * X)) $P tests/test_gpu_sighash.py \
      -k multisig_block_stress > ${O}_multisig.log 2>&1 && echo "multisig ok" \
    && HKV_STRESS_MS_BLOCKS=$((24 * X)) HKV_STRESS_MS_WINDOW=256,64 timeout -k 10 $((400 * X)) $P \
      tests/test_gpu_sighash.py -k multisig_block_stress > ${O}_multisig_rounds.log 2>&1 && echo "multisig rounds ok" \
    && HKV_STRESS_ROUNDS=$((400 * X)) timeout -k 10 $((200 * X)) $P tests/test_gpu_concurrency.py \
      > ${O}_concurrency.log 2>&1 && echo "concurrency ok"
  ;;
*)
  echo "unknown mode $MODE" >&2
  exit 2
  ;;
esac
