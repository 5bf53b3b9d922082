#!/bin/bash
# Branch-free safegcd divsteps (HKV_SGCD_FLAT): the GPU suite on the in-tree
# (flat) build, then flat / branchy benches alternating, then the
# signature-wave stamp builds of both (s^-1 time).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05v_pytest.log 2>&1 \
  && tail -1 gpurun_out/r05v_pytest.log || exit 1
VARIANTS="flat noflat flat noflat st4flat st4noflat" BENCH_ARGS="--no-adversarial --no-headers --no-merkle --no-host-path --no-inproc" \
  bash tools/variants.sh || exit 1
for v in st4flat st4noflat; do
  python3 - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/variant_{v}.log").read().strip().splitlines()[-1])
for leg, x in (("c0", d["config0"]), ("c2", d["block_mix"]["block"])):
    p = x["split_phases_us"]
    print(v, leg, x["total_us"], {k: p[k] for k in ("lo_table", "hi_table", "digits", "key_sqrt", "sig_parse", "lo_chain", "verdict")})
PY
done
