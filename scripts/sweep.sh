#!/bin/bash
# generic bench sweep: every line of $CONFIGS (bench.py arguments) once per repetition;
# prints value, ms/step and per-stage ms for each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/sweep${TAG}
mkdir -p $OUT
i=0
while read -r args; do
  [ -z "$args" ] && continue
  i=$((i+1))
  for rep in $(seq ${REPS:-1}); do
    timeout -k 10 300 python bench.py --steps ${STEPS:-60} --warmup 5 --no-cpu $args > $OUT/c${i}_r${rep}.json 2>>$OUT/err.log
    rc=$?; [ $rc -ge 124 ] && exit $rc
    python3 -c "import json,sys;d=json.load(open('$OUT/c${i}_r${rep}.json'));print('$args'.ljust(40), d['value'], d['ms_per_step'], (d['roofline'] or {}).get('stages_ms'))"
  done
done <<< "$CONFIGS"
