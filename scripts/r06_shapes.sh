#!/bin/bash
# round 6: the three per-rank slabs of the driver's N = 8 / 4 / 2 cube workloads (400x400x100, 318x318x159,
# 252x252x252 cells), bench.py --steps 100 on one MI355X: one slab with no exchange (plain), the self
# exchange over the put-kernel ipc (ipc), over ipc-ce (ce = the default placement, ceN = PFT_CE_BND=N: 0 every
# boundary launch before its interior); $EXTRA is added to every run, $VARS / $SHAPES select.
# Output gpurun_out/shapes$TAG; prints value, ms/step, per-stage ms, pair tile and z-chunk planes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/shapes${TAG}
mkdir -p $OUT
for rep in $(seq ${REPS:-2}); do
  for dom in ${SHAPES:-"400:0.06,0.06,0.015:n8" "318:0.06,0.06,0.03:n4" "252:0.06,0.06,0.06:n2"}; do
    IFS=: read nodes domain name <<< "$dom"
    for v in ${VARS:-plain ipc ce ce0}; do
      args="--steps 100 --warmup 5 --no-cpu --grid-nodes $nodes --domain $domain $EXTRA"
      f=$OUT/${name}_${v}_$rep.json
      case $v in
        plain) timeout -k 10 300 python bench.py $args > $f 2>>$OUT/err.log ;;
        ipc) timeout -k 10 300 python bench.py $args --self-exchange --transport ipc > $f 2>>$OUT/err.log ;;
        ce) timeout -k 10 300 python bench.py $args --self-exchange --transport ipc-ce > $f 2>>$OUT/err.log ;;
        ce0) PFT_CE_BND=0 timeout -k 10 300 python bench.py $args --self-exchange --transport ipc-ce > $f 2>>$OUT/err.log ;;
        ce4) PFT_CE_BND=4 timeout -k 10 300 python bench.py $args --self-exchange --transport ipc-ce > $f 2>>$OUT/err.log ;;
        ce5) PFT_CE_BND=5 timeout -k 10 300 python bench.py $args --self-exchange --transport ipc-ce > $f 2>>$OUT/err.log ;;
        ce3) PFT_CE_BND=3 timeout -k 10 300 python bench.py $args --self-exchange --transport ipc-ce > $f 2>>$OUT/err.log ;;
      esac
      rc=$?; [ $rc -ne 0 ] && { echo "$name $v failed: $rc"; exit $rc; }
      python3 -c "import json;d=json.load(open('$f'));print('$name $v rep $rep'.ljust(20), d['value'], d['ms_per_step'], (d['roofline'] or {}).get('stages_ms'), d['config'].get('pair_tile'))"
    done
  done
done
