#!/bin/bash
# A/B of the library builds in $LIBS (porousfreezethaw_amd/<dir>/libpft.so): the pair-kernel
# parity tests on each non-default build, then the bench at $STEPS steps, $REPS interleaved rounds.
# Outputs under gpurun_out/abq/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/abq
mkdir -p $O
for lib in ${LIBS:-lib lib_alt}; do
  [ "$lib" = lib ] && continue
  PFT_LIB=$PWD/porousfreezethaw_amd/$lib/libpft.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${TESTS:-tests/test_pair_gpu.py} > $O/pytest_$lib.log 2>&1 || { echo "$lib: pytest failed"; tail -30 $O/pytest_$lib.log; exit 1; }
  echo "$lib: $(tail -1 $O/pytest_$lib.log)"
done
for rep in $(seq ${REPS:-2}); do
  for lib in ${LIBS:-lib lib_alt}; do
    PFT_LIB=$PWD/porousfreezethaw_amd/$lib/libpft.so timeout -k 10 300 python bench.py --steps ${STEPS:-200} --warmup 10 --no-cpu $ARGS > $O/${lib}_r${rep}.json 2>>$O/err.log || { echo "$lib bench failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${lib}_r${rep}.json'));print('$lib'.ljust(10), d['value'], d['ms_per_step'], (d['roofline'] or {}).get('stages_ms'))"
  done
done
