#!/usr/bin/env python3
"""The distinct `icond` formula sets of the reference's published cases -> tests/golden/icond_published.json.

Test infrastructure only: reads the Params files inside the reference's results/ archives and its
default Params (apps/intertrack-hybrid-S-freezing) as text and stores the formula strings (data:
the three icond lines of each distinct case, with how many of the 86 published cases use them), so
that the GPU test of the device IC (tests/test_device_ic.py), which runs where /root/reference
does not exist, evaluates the published formulas.  Re-run with:  python tests/golden/gen_icond.py
"""
import glob
import json
import os
import re
import tarfile

APP = "/root/reference/apps/intertrack-hybrid-S-freezing"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "icond_published.json")


def icond_of(text):
    f = {}
    for line in text.splitlines():
        m = re.match(r'\s*icond\s+(\w+)\s*=\s*"([^"]*)"', line)
        if m:
            f[m.group(1)] = m.group(2)
    return f


def main():
    sets, counts = [], []
    for arc in sorted(glob.glob(os.path.join(APP, "results", "*", "*.tgz"))):
        with tarfile.open(arc) as tf:
            for m in tf.getmembers():
                if m.isfile() and m.name.endswith("/Params"):
                    f = icond_of(tf.extractfile(m).read().decode("latin-1"))
                    if len(f) != 3:
                        continue
                    if f in sets:
                        counts[sets.index(f)] += 1
                    else:
                        sets.append(f)
                        counts.append(1)
    default = icond_of(open(os.path.join(APP, "Params"), encoding="latin-1").read())
    out = {"source": "icond lines of apps/intertrack-hybrid-S-freezing/Params and of the Params in its "
                     "results/*/*.tgz archives (tests/golden/gen_icond.py)",
           "default": default,
           "published": [{"cases": c, "icond": f} for f, c in zip(sets, counts)]}
    with open(OUT, "w") as fh:
        json.dump(out, fh, indent=1)
    print(f"{len(sets)} distinct formula sets over {sum(counts)} published cases -> {OUT}")


if __name__ == "__main__":
    main()
