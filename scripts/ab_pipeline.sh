#!/bin/bash
# N > 1 stage-pipeline orders on one GPU (1-rank RCCL self-exchange rehearsal) on the per-rank
# slabs of the 800^3 8-way and 636^3 4-way cubes: one-stream (default) vs comm-boundary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/abpipe; mkdir -p $O
for rep in 1 2; do
  for dom in "400 0.06,0.06,0.015 n8" "318 0.06,0.06,0.03 n4"; do
    set -- $dom
    for v in one comm; do
      extra=""; [ $v = comm ] && extra="--comm-boundary"
      timeout -k 10 200 python bench.py --steps 100 --no-cpu --grid-nodes $1 --domain $2 --self-exchange $extra > $O/${3}_${v}_r${rep}.json 2>>$O/err.log || { echo "fail $3 $v"; exit 1; }
      python3 -c "import json;d=json.load(open('$O/${3}_${v}_r${rep}.json'));print('$3 $v', d['value'], d['ms_per_step'])"
    done
  done
done
