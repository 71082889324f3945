#!/bin/bash
# pair kernels on / off (PFT_PAIR) over the bench workloads of SURVEY 8(d) on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/abcfg${TAG}
mkdir -p $OUT
while read -r label args; do
  [ -z "$label" ] && continue
  for pair in 1 0; do
    PFT_PAIR=$pair timeout -k 10 300 python bench.py --no-cpu $args > $OUT/${label}_p$pair.json 2>>$OUT/err.log
    rc=$?; [ $rc -ne 0 ] && { echo "$label failed: $rc"; exit $rc; }
    python3 -c "import json;d=json.load(open('$OUT/${label}_p$pair.json'));print('$label p$pair'.ljust(16), d['value'], d['ms_per_step'], (d['roofline'] or {}).get('stages_ms'))"
  done
done <<< "${CONFIGS:-default --steps 100
g200 --steps 400 --grid-nodes 200
g100 --steps 2000 --warmup 20 --grid-nodes 100
mode1 --steps 100 --mode 1
mode2 --steps 100 --mode 2
gls --steps 100 --gl-static
cube --steps 30 --literal-cube
slab8 --steps 100 --grid-nodes 400 --domain 0.06,0.06,0.015
slab4 --steps 100 --grid-nodes 318 --domain 0.06,0.06,0.03
slab2 --steps 100 --grid-nodes 252 --domain 0.06,0.06,0.06}"
