#!/usr/bin/env python3
"""Summarise rocprofv3 runs of bench.py into profiles/pmc_summary.json.

Inputs (directories written by scripts/evidence.sh): a kernel-trace/--stats run and two PMC
runs (FETCH_SIZE, WRITE_SIZE -- separate passes, MI355X_MICROARCH.md "rocprofv3 PMC slots").
Corrections (MI355X_MICROARCH.md "HBM"): FETCH_SIZE/WRITE_SIZE are in KiB; gfx950's FETCH_SIZE
is only exact for calibrated access widths, so the ratio known/measured of the probe_copy_kernel
(8-byte loads and stores per lane, exactly the stage kernels' width, known byte count) calibrates
both counters.  Output keys: stage<k>_gl<0|1>_<n1>x<n2>x<n3>_m<mode> (the slab's cells; pair<k> for
the pair kernel whose second stage is k) -> HBM bytes per launch.  With a fourth run (SQ_INSTS_VALU
and GRBM_GUI_ACTIVE in one pass), also the VALU issue fraction per kernel:
  SQ_INSTS_VALU x 4 cycles (a wave64 VALU instruction on a 16-lane SIMD) / (1024 SIMDs x the
  kernel's cycles, GRBM_GUI_ACTIVE / 8 XCDs) = SQ_INSTS_VALU / (32 GRBM_GUI_ACTIVE).
With a fifth run (SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 and GRBM_GUI_ACTIVE in one pass,
scripts/pmc_fp64.sh), the FP64 work per launch: FLOP = 64 lanes x (ADD + MUL + TRANS + 2 FMA)
wave instructions, and the FP64 pipe's busy fraction = 4 cycles per wave64 FP64 instruction (16
FP64 lanes per SIMD and cycle: the 78.6 TFLOP/s vector peak) / (1024 SIMDs x the kernel's cycles).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def rows(d, pattern):
    out = []
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def counters(d, name):
    acc = defaultdict(list)
    for r in rows(d, "*counter_collection.csv"):
        if r.get("Counter_Name") != name:
            continue
        acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def kname(k):
    m = re.search(r"merson_(?:stage|tile|fused)<(\d+),\s*(\d+),\s*(true|false)", k)
    if m:
        return f"stage{m.group(1)}", m.group(2), m.group(3) == "true"
    m = re.search(r"merson_pair<(\d+),\s*(\d+),\s*(true|false)", k)
    if m:
        return f"pair{int(m.group(1)) + 1}", m.group(2), m.group(3) == "true"
    if "probe_copy" in k:
        return "probe", None, None
    return None, None, None


def main(trace_dir, fetch_dir, write_dir, dims, probe_bytes, out_path, valu_dir=None, fp64_dir=None):
    fetch, write = counters(fetch_dir, "FETCH_SIZE"), counters(write_dir, "WRITE_SIZE")
    f64 = {c: counters(fp64_dir, "SQ_INSTS_VALU_" + c + "_F64") for c in ("ADD", "MUL", "FMA", "TRANS")} if fp64_dir else {}
    grbm64 = counters(fp64_dir, "GRBM_GUI_ACTIVE") if fp64_dir else {}
    valu = counters(valu_dir, "SQ_INSTS_VALU") if valu_dir else {}
    grbm = counters(valu_dir, "GRBM_GUI_ACTIVE") if valu_dir else {}
    pf = [v for k, v in fetch.items() if kname(k)[0] == "probe"]
    pw = [v for k, v in write.items() if kname(k)[0] == "probe"]
    cal_f = probe_bytes / (pf[0] * 1024) if pf else 1.0
    cal_w = probe_bytes / (pw[0] * 1024) if pw else 1.0
    stats = {}
    for r in rows(trace_dir, "*kernel_stats.csv"):
        stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                            "pct": float(r.get("Percentage", 0))}
    res = {"calibration": {"probe_bytes": probe_bytes, "fetch_factor": cal_f, "write_factor": cal_w,
                           "probe_FETCH_SIZE_KiB": pf[0] if pf else None,
                           "probe_WRITE_SIZE_KiB": pw[0] if pw else None}}
    for k in set(fetch) | set(write):
        st, mode, gls = kname(k)
        if not st or st == "probe":
            continue
        fb = fetch.get(k, 0.0) * 1024 * cal_f
        wb = write.get(k, 0.0) * 1024 * cal_w
        # a pair kernel's third template parameter is GLX (gl_static or gl_keep), a stage kernel's GLS
        key = f"{st}_{'glx' if st.startswith('pair') else 'gl'}{int(gls)}_{dims}_m{mode}"
        res[key] = {"kernel": k, "fetch_bytes": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb,
                    "raw_FETCH_SIZE_KiB": fetch.get(k), "raw_WRITE_SIZE_KiB": write.get(k)}
        if k in valu and grbm.get(k):
            res[key]["SQ_INSTS_VALU"] = valu[k]
            res[key]["GRBM_GUI_ACTIVE"] = grbm[k]
            res[key]["valu_issue_frac"] = valu[k] / (32.0 * grbm[k])
        if f64 and all(k in f64[c] for c in f64) and grbm64.get(k):
            ins = {c: f64[c][k] for c in f64}
            n = ins["ADD"] + ins["MUL"] + ins["FMA"] + ins["TRANS"]
            res[key]["fp64_wave_insts"] = ins
            res[key]["fp64_flop_per_launch"] = 64.0 * (n + ins["FMA"])
            res[key]["fp64_pipe_busy_frac"] = 4.0 * n / (1024.0 * grbm64[k] / 8.0)
    res["kernel_stats"] = stats
    # where these numbers come from (bench.py copies this into roofline.traffic_source)
    res["provenance"] = {"tool": "rocprofv3 --pmc FETCH_SIZE, --pmc WRITE_SIZE and --pmc SQ_INSTS_VALU "
                                 "GRBM_GUI_ACTIVE, --pmc SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 GRBM_GUI_ACTIVE, "
                                 "separate passes of bench.py (scripts/evidence.sh); "
                                 "FETCH_SIZE x fetch_factor from the probe copy",
                         "tag": os.environ.get("TAG", ""),
                         "date": os.environ.get("PMC_DATE", ""),
                         "git": os.environ.get("PMC_GIT", "")}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps({k: v.get("hbm_bytes_per_launch") for k, v in res.items() if isinstance(v, dict)}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5]), sys.argv[6],
         sys.argv[7] if len(sys.argv) > 7 else None, sys.argv[8] if len(sys.argv) > 8 else None)
