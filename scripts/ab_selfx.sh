#!/bin/bash
# per-rank slabs of the N > 1 cube workloads on one GPU: plain, and through the N > 1 path of each
# transport with a self-exchanging 1-rank communicator (bench.py --self-exchange); $PAIRS = the
# PFT_PAIR values to compare
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/selfx${TAG}
mkdir -p $OUT
for dom in "400 0.06,0.06,0.015 n8" "318 0.06,0.06,0.03 n4" "252 0.06,0.06,0.06 n2"; do
  set -- $dom
  for pair in ${PAIRS:-1 0}; do
    for tr in none ipc rccl; do
      args="--steps 100 --no-cpu --grid-nodes $1 --domain $2"
      [ $tr != none ] && args="$args --self-exchange --transport $tr"
      PFT_PAIR=$pair timeout -k 10 300 python bench.py $args > $OUT/$3_p${pair}_$tr.json 2>>$OUT/err.log
      rc=$?; [ $rc -ne 0 ] && { echo "$3 $tr failed: $rc"; exit $rc; }
      python3 -c "import json;d=json.load(open('$OUT/$3_p${pair}_$tr.json'));print('$3 p$pair $tr'.ljust(14), d['value'], d['ms_per_step'], (d['roofline'] or {}).get('stages_ms'))"
    done
  done
done
