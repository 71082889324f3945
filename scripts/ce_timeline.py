"""Timeline of a rocprofv3 --kernel-trace --memory-copy-trace run (the copy-engine exchange): kernels and
SDMA copies around one launch of a kernel, times in us relative to that launch's start.
usage: python scripts/ce_timeline.py <trace dir> [kernel: pair4|pair2|fused1] [which: -3]"""
import csv, glob, sys

d = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else "pair4"
which = int(sys.argv[3]) if len(sys.argv) > 3 else -3
ev = []
for r in csv.DictReader(open(glob.glob(d + "/*kernel_trace.csv")[0])):
    n = r["Kernel_Name"]
    s = ("pair4" if "merson_pair<4" in n else "pair2" if "merson_pair<2" in n else
         "fused" + n.split("merson_fused<")[1][0] if "merson_fused<" in n else
         "trig" if "bnd_trigger" in n else "wait" if "halo_wait" in n else n[:24])
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), s, "grid " + r["Grid_Size_X"]))
for r in csv.DictReader(open(glob.glob(d + "/*memory_copy_trace.csv")[0])):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy", "stream " + r["Stream_Id"]))
ev.sort()
idx = [i for i, e in enumerate(ev) if e[2] == want]
i = idx[which]
t0 = ev[i][0]
for e in ev[max(0, i - 12):i + 25]:
    print(f"{(e[0] - t0) / 1000:9.1f} {(e[1] - t0) / 1000:9.1f} {(e[1] - e[0]) / 1000:8.1f}  {e[2]:8s} {e[3]}")
