#!/bin/bash
# Round 4 kernel A/B: $TESTS on lib/ first (stop on failure), then for each argument set in $CASES
# (one per line: label|bench args|env) the libraries in $LIBS interleaved over $REPS rounds.
# Outputs under gpurun_out/ab4${TAG}/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/ab4${TAG}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider $TESTS > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { tail -40 $O/pytest.log; exit $rc; }
fi
i=0
while IFS='|' read -r label args envs; do
  [ -z "$label" ] && continue
  i=$((i+1))
  for rep in $(seq ${REPS:-2}); do
    for lib in ${LIBS:-lib lib_alt}; do
      env $envs PFT_LIB=$PWD/porousfreezethaw_amd/$lib/libpft.so timeout -k 10 300 python bench.py --no-cpu $args > $O/c${i}_${lib}_r${rep}.json 2>>$O/err.log
      rc=$?; [ $rc -ne 0 ] && { echo "$label $lib failed: $rc"; tail -5 $O/err.log; exit $rc; }
      python3 -c "import json;d=json.load(open('$O/c${i}_${lib}_r${rep}.json'));print('$label'.ljust(14), '$lib'.ljust(9), d['value'], d['ms_per_step'], (d['roofline'] or {}).get('stages_ms'))"
    done
  done
done <<< "$CASES"
