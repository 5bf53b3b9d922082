"""Per-kernel VGPRs / spills / occupancy / LDS of hkv_kernels.hip (or another
HIP source) from clang's -Rpass-analysis=kernel-resource-usage remarks.
Usage: python tools/resource_usage.py [source.hip] [extra hipcc flags...]"""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "haskoin-node_amd/csrc/hkv_kernels.hip"
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-x", "hip", "-c", src, "-o", "/dev/null",
       "--cuda-device-only", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]|ScratchSize \[bytes/lane\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt"], input=v, capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k.split(" [")[0]] = v
for r in rows:
    print(f"{r['name'][:70]:70s} vgpr={r.get('VGPRs','?'):>4} spill={r.get('VGPRs Spill','?'):>4} "
          f"scratch={r.get('ScratchSize','?'):>5} occ={r.get('Occupancy','?'):>2} lds={r.get('LDS Size','?')}")
