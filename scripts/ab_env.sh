#!/bin/bash
# A/B of environment / library variants on one box.  Each line of $CASES is
# "<label> <lib dir> <env assignments...>"; every case runs bench.py (default workload plus $ARGS)
# $REPS times, interleaved; prints value, ms/step and per-stage ms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/abenv${TAG}
mkdir -p $OUT
for rep in $(seq ${REPS:-1}); do
  while read -r label lib envs; do
    [ -z "$label" ] && continue
    env $envs PFT_LIB=$PWD/porousfreezethaw_amd/$lib/libpft.so timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup 5 --no-cpu $ARGS > $OUT/${label}_r${rep}.json 2>>$OUT/err.log
    rc=$?; [ $rc -ne 0 ] && { echo "$label failed: $rc"; exit $rc; }
    python3 -c "import json;d=json.load(open('$OUT/${label}_r${rep}.json'));print('$label'.ljust(14), d['value'], d['ms_per_step'], (d['roofline'] or {}).get('stages_ms'))"
  done <<< "$CASES"
done
