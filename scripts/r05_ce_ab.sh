#!/bin/bash
# round 5: the copy-engine exchange's options on the 800^3 rank slab (self exchange, 100 steps):
# PFT_CE_BND (0 boundary launch before the interior, 1 beside it for every launch, 2 beside it for
# the pair kernels, 3 the boundary pipeline) x PFT_CE_STREAMS (1 or 2 copy streams; 4 was removed);
# $REPS repetitions, output gpurun_out/ceab$TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/ceab${TAG}
mkdir -p $OUT
args="--steps ${STEPS:-100} --no-cpu --grid-nodes 400 --domain 0.06,0.06,0.015"
for rep in ${REPS:-1}; do
  for v in ${VARS:-none 0,2 2,2 3,2}; do
    if [ $v = none ]; then
      timeout -k 10 300 python bench.py $args > $OUT/${v}_$rep.json 2>>$OUT/err.log
    else
      PFT_CE_BND=${v%,*} PFT_CE_STREAMS=${v#*,} timeout -k 10 300 python bench.py $args --self-exchange --transport ipc-ce > $OUT/${v}_$rep.json 2>>$OUT/err.log
    fi
    rc=$?; [ $rc -ne 0 ] && { echo "$v failed: $rc"; exit $rc; }
    python3 -c "import json;d=json.load(open('$OUT/${v}_$rep.json'));print('bnd,streams $v rep $rep'.ljust(24), d['value'], d['ms_per_step'], (d['roofline'] or {}).get('stages_ms'))"
  done
done
