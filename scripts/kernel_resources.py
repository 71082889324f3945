#!/usr/bin/env python3
"""Per-kernel VGPR / spill / occupancy table of pft_kernels.hip for gfx950 (compiler remarks).

    python scripts/kernel_resources.py [filter-regex] [extra hipcc flags...]
"""
import re
import subprocess
import sys

flt = re.compile(sys.argv[1] if len(sys.argv) > 1 else "merson_fused")
extra = sys.argv[2:]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off",
       "-fno-fast-math", "-Wno-unused-result", "-c", __import__("os").environ.get("PFT_SRC","porousfreezethaw_amd/csrc/pft_kernels.hip"), "-o",
       "/tmp/pft_kernels_res.o", "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        dm = subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()
        cur = {"name": dm.split("(")[0]}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if flt.search(r["name"]):
        print(f"{r['name']:48s} vgpr {r.get('VGPRs','?'):>4s} vspill {r.get('VGPRs Spill','?'):>3s} "
              f"sspill {r.get('SGPRs Spill','?'):>3s} occ {r.get('Occupancy [waves/SIMD]','?'):>2s} "
              f"lds {r.get('LDS Size [bytes/block]','?')}")
