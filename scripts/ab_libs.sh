#!/bin/bash
# A/B of library builds on one box: the default bench workload (plus $ARGS) on every library in
# $LIBS (directories under porousfreezethaw_amd/, built with make OBJ=build_X LIBDIR=lib_X
# EXTRA=-D...), $REPS rounds interleaved; prints value, ms/step and per-stage ms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/ab${TAG}
mkdir -p $OUT
for rep in $(seq ${REPS:-2}); do
  for lib in ${LIBS:-lib lib_alt}; do
    PFT_LIB=$PWD/porousfreezethaw_amd/$lib/libpft.so timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup 5 --no-cpu $ARGS > $OUT/${lib}_r${rep}.json 2>>$OUT/err.log
    rc=$?; [ $rc -ne 0 ] && { echo "$lib failed: $rc"; exit $rc; }
    python3 -c "import json;d=json.load(open('$OUT/${lib}_r${rep}.json'));print('$lib'.ljust(10), d['value'], d['ms_per_step'], (d['roofline'] or {}).get('stages_ms'))"
  done
done
