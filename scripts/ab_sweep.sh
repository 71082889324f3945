#!/bin/bash
# A/B of library builds (lib vs lib_alt) over kz, one process per run, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
PFT_LIB=$PWD/porousfreezethaw_amd/lib_alt/libpft.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider -k "trajectory or oracle or loopback" > gpurun_out/ab/pytest_alt.log 2>&1; tail -1 gpurun_out/ab/pytest_alt.log
for lib in lib lib_alt; do
  for kz in ${KZS:-8 16 25 32}; do
    for gls in "" "--gl-static"; do
      PFT_LIB=$PWD/porousfreezethaw_amd/$lib/libpft.so timeout -k 10 300 python bench.py --steps 60 --warmup 5 --no-cpu --kz $kz --tile ${TILE:-16} $gls > gpurun_out/ab/${lib}_kz${kz}${gls}.json 2>>gpurun_out/ab/err.log
      rc=$?; [ $rc -ge 124 ] && exit $rc
    done
  done
done
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/ab/lib*.json")):
    try: d = json.load(open(f))
    except Exception as e: print(f, "ERR", e); continue
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d["roofline"]["stages_ms"])
PY
