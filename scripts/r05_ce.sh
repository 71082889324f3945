#!/bin/bash
# round 5: the copy-engine ipc exchange on the 800^3 rank slab (400x400x100), self exchange, against
# plain, the put-kernel ipc and RCCL; $TRS = transports, $TAG = output suffix
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/ce${TAG}
mkdir -p $OUT
for rep in ${REPS:-1}; do
  for tr in ${TRS:-none ipc-ce ipc rccl}; do
    args="--steps ${STEPS:-100} --no-cpu --grid-nodes 400 --domain 0.06,0.06,0.015"
    [ $tr != none ] && args="$args --self-exchange --transport $tr"
    timeout -k 10 300 python bench.py $args > $OUT/n8_${tr}_$rep.json 2>>$OUT/err.log
    rc=$?; [ $rc -ne 0 ] && { echo "$tr failed: $rc"; exit $rc; }
    python3 -c "import json;d=json.load(open('$OUT/n8_${tr}_$rep.json'));print('n8 $tr $rep'.ljust(16), d['value'], d['ms_per_step'], (d['roofline'] or {}).get('stages_ms'))"
  done
done
