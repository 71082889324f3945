#!/bin/bash
# A/B of library builds (LIBS, default "lib lib_alt") over kz, one process per run, same box.
#   KZS="8 16"  TILE=32  REPS=2  GLS="0 1"  NOTEST=1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
if [ -z "$NOTEST" ]; then
  PFT_LIB=$PWD/porousfreezethaw_amd/lib_alt/libpft.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider -k "trajectory or oracle or loopback" > gpurun_out/ab/pytest_alt.log 2>&1; tail -1 gpurun_out/ab/pytest_alt.log
fi
for rep in $(seq ${REPS:-1}); do
for lib in ${LIBS:-lib lib_alt}; do
  for kz in ${KZS:-8 16 25 32}; do
    for gls in ${GLS:-0 1}; do
      flag=""; [ "$gls" = 1 ] && flag="--gl-static"
      PFT_LIB=$PWD/porousfreezethaw_amd/$lib/libpft.so timeout -k 10 300 python bench.py --steps ${STEPS:-60} --warmup 5 --no-cpu --kz $kz --tile ${TILE:-16} $flag > gpurun_out/ab/${lib}_kz${kz}_gls${gls}_r${rep}.json 2>>gpurun_out/ab/err.log
      rc=$?; [ $rc -ge 124 ] && exit $rc
    done
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
