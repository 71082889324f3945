#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/sweep
for tile in ${TILES:-0 16 32}; do
  for kz in ${KZS:-4 8 16}; do
    for gls in "" "--gl-static"; do
      timeout -k 10 300 python bench.py --steps 60 --warmup 5 --no-cpu --kz $kz --tile $tile $gls > gpurun_out/sweep/t${tile}_kz${kz}${gls}.json 2>>gpurun_out/sweep/err.log
      rc=$?; [ $rc -ge 124 ] && exit $rc
    done
  done
done
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/sweep/t*.json")):
    try: d = json.load(open(f))
    except Exception as e: print(f, "ERR", e); continue
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["roofline"]["stages_ms"])
PY
