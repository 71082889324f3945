#!/bin/bash
# round 5: the copy-engine exchange's boundary placement on the three per-rank slabs of the driver's
# N = 2 / 4 / 8 cube workloads (self exchange, 100 steps): PFT_CE_BND 0 (boundary launch before the
# interior) against 2 (the pair kernels' beside it), beside the put-kernel ipc; output gpurun_out/ceshape$TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/ceshape${TAG}
mkdir -p $OUT
for rep in ${REPS:-1}; do
  for dom in "400 0.06,0.06,0.015 n8" "318 0.06,0.06,0.03 n4" "252 0.06,0.06,0.06 n2"; do
    set -- $dom
    for v in ${VARS:-ipc 0 2 3}; do
      args="--steps 100 --no-cpu --grid-nodes $1 --domain $2 --self-exchange"
      if [ $v = ipc ]; then
        timeout -k 10 300 python bench.py $args --transport ipc > $OUT/$3_${v}_$rep.json 2>>$OUT/err.log
      else
        PFT_CE_BND=$v timeout -k 10 300 python bench.py $args --transport ipc-ce > $OUT/$3_${v}_$rep.json 2>>$OUT/err.log
      fi
      rc=$?; [ $rc -ne 0 ] && { echo "$3 $v failed: $rc"; exit $rc; }
      python3 -c "import json;d=json.load(open('$OUT/$3_${v}_$rep.json'));print('$3 $v rep $rep'.ljust(18), d['value'], d['ms_per_step'], (d['roofline'] or {}).get('stages_ms'))"
    done
  done
done
