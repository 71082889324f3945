"""Timeline of the last attempted steps of a rocprofv3 --kernel-trace --memory-copy-trace run (csv):
every kernel and copy with its stream, start and end in microseconds from the first listed event.
Usage: python scripts/ce_timeline.py <dir with run_kernel_trace.csv> [n_events]"""
import csv
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
ev = []
for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
    name = r["Kernel_Name"]
    name = name.split("(")[0][:60]
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Stream_Id"], name, r["Grid_Size_X"]))
p = os.path.join(d, "run_memory_copy_trace.csv")
if os.path.exists(p):
    for r in csv.DictReader(open(p)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", r["Stream_Id"], r["Direction"], ""))
ev.sort()
ev = ev[-n:]
t0 = ev[0][0]
for s, e, k, st, name, g in ev:
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  {k} s{st:>3} {name} {g}")
