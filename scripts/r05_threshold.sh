#!/bin/bash
# the pair kernels' size threshold (4 Ki cells per CU, ~1.05 M cells on 256 CUs) between
# the measured 100^3 (1 Ki/CU) and 200^3 (7.8 Ki/CU): grid_nodes 110, 128, 160 with the pair kernels
# forced on (PFT_PAIR=2) and off (PFT_PAIR=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/thr
mkdir -p $OUT
for g in ${GS:-110 128 160}; do
  for pair in 0 2; do
    PFT_PAIR=$pair timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu --grid-nodes $g > $OUT/g${g}_p$pair.json 2>>$OUT/err.log || exit 1
    python3 -c "import json;d=json.load(open('$OUT/g${g}_p$pair.json'));c=d['config'];print('g$g pair=$pair', c['cells'], d['value'], d['ms_per_step'], c['pair_kernels'])"
  done
done
