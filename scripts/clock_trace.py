#!/usr/bin/env python3
"""Effective GPU clock per kernel launch from a rocprofv3 --pmc GRBM_GUI_ACTIVE pass
(scripts/quick.sh with CLOCK=1): GRBM_GUI_ACTIVE is summed over the 8 XCDs, so the clock of a
dispatch is GRBM_GUI_ACTIVE / 8 / (End - Start).  Shows that the slow first launches of a short
bench run run at a lower clock with the same cycle count (GPU power management ramping up), not
more work.

    python scripts/clock_trace.py gpurun_out/q/clk/run_counter_collection.csv [kernel-substring]
"""
import collections
import csv
import sys

path = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else "merson"
d = collections.OrderedDict()
for r in csv.DictReader(open(path)):
    k = int(r["Dispatch_Id"])
    e = d.setdefault(k, {"name": r["Kernel_Name"].split("(")[0].replace("void ", ""),
                         "t0": int(r["Start_Timestamp"]), "t1": int(r["End_Timestamp"])})
    e[r["Counter_Name"]] = float(r["Counter_Value"])
first = None
print(f"{'dispatch':>8} {'t (ms)':>8} {'us':>8} {'Mcycles/XCD':>12} {'GHz':>6}  kernel")
for k, e in d.items():
    if flt not in e["name"] or "GRBM_GUI_ACTIVE" not in e:
        continue
    first = e["t0"] if first is None else first
    us = (e["t1"] - e["t0"]) / 1e3
    cyc = e["GRBM_GUI_ACTIVE"] / 8.0
    print(f"{k:8d} {(e['t0'] - first) / 1e6:8.3f} {us:8.1f} {cyc / 1e6:12.4f} {cyc / us / 1e3:6.3f}  {e['name']}")
