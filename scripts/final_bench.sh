#!/bin/bash
# The default bench line (with cpu_baseline) and the driver's configuration three times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/fb
mkdir -p $O
timeout -k 10 400 python bench.py > $O/default.json 2> $O/default.err || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu > $O/driver_$r.json 2>> $O/err.log || exit 1
done
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/fb/default.json"))
print("default", d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["stages_ms"], d["cpu_baseline"]["value"])
for r in (1, 2, 3):
    e = json.load(open(f"gpurun_out/fb/driver_{r}.json"))
    print("driver cfg", e["value"], e["ms_per_step"])
PY
