#!/usr/bin/env python3
"""Per-step timeline of a rocprofv3 kernel trace (one process, one stream of stage kernels):
median duration of each kernel kind and of the gap before it, and the step period.
usage: step_timeline.py run_kernel_trace.csv [first_kernels_to_skip]"""
import collections
import csv
import re
import statistics as st
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 50
rows = rows[skip:]


def kind(r):
    n = r["Kernel_Name"]
    m = re.search(r"(merson_\w+)<(\d+)", n)
    if m:
        return f"{m.group(1)}<{m.group(2)}> grid {r['Grid_Size_X']}"
    return n.split("(")[0][:40]


dur, gap = collections.defaultdict(list), collections.defaultdict(list)
for a, b in zip(rows, rows[1:]):
    k = kind(b)
    dur[k].append((int(b["End_Timestamp"]) - int(b["Start_Timestamp"])) / 1e3)
    gap[k].append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
print(f"{'kernel':58s} {'n':>6s} {'dur us':>8s} {'gap before':>10s}")
for k in sorted(dur, key=lambda k: -len(dur[k])):
    print(f"{k:58s} {len(dur[k]):6d} {st.median(dur[k]):8.2f} {st.median(gap[k]):10.2f}")
pub = [int(r["Start_Timestamp"]) for r in rows if r["Kernel_Name"].startswith("publish_kernel")]
if len(pub) > 2:
    per = [(b - a) / 1e3 for a, b in zip(pub, pub[1:])]
    print(f"step period (publish to publish): median {st.median(per):.2f} us, mean {st.mean(per):.2f} us")
