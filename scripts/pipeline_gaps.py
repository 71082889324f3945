#!/usr/bin/env python3
"""Per-stage timeline of the N > 1 stage pipeline from a rocprofv3 kernel trace (scripts/pipeline_trace.sh):
boundary-launch duration, the gap to the interior sweep, the interior duration, the gap to the next
boundary launch, and the RCCL kernel durations.  usage: pipeline_gaps.py run_kernel_trace.csv"""
import csv
import statistics as st
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
fused = [r for r in rows if "merson_fused" in r["Kernel_Name"]]
rccl = [r for r in rows if "nccl" in r["Kernel_Name"].lower()]
grids = sorted({int(r["Grid_Size_X"]) for r in fused})
small = grids[0]                      # the boundary launch: two one-plane chunks
bnd_ms, gap_bi, gap_ib = [], [], []
for a, b in zip(fused, fused[1:]):
    ga, gb = int(a["Grid_Size_X"]), int(b["Grid_Size_X"])
    s0, e0, s1 = int(a["Start_Timestamp"]), int(a["End_Timestamp"]), int(b["Start_Timestamp"])
    if ga == small and gb != small:
        bnd_ms.append((e0 - s0) / 1e3)
        gap_bi.append((s1 - e0) / 1e3)
    elif ga != small and gb == small:
        gap_ib.append((s1 - e0) / 1e3)


def q(v):
    v = sorted(v)
    return f"n={len(v)} median {st.median(v):.1f} us, p10 {v[len(v) // 10]:.1f}, p90 {v[9 * len(v) // 10]:.1f}"


print("boundary launch duration:", q(bnd_ms))
print("gap boundary -> interior:", q(gap_bi))
print("gap interior -> next boundary (exchange wait):", q(gap_ib))
print("RCCL kernels:", q([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rccl]))
