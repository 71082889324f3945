#!/bin/bash
# f4 (small slabs): 100^3 and 200^3 with the stage launches and with the pair kernels forced
# (PFT_PAIR=2), bench lines and one kernel trace each.  Outputs under gpurun_out/sg/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/sg
mkdir -p $O
[ -n "$LIBDIR" ] && export PFT_LIB=$PWD/porousfreezethaw_amd/$LIBDIR/libpft.so
for g in 100 200; do
  st=$([ $g = 100 ] && echo 2000 || echo 400)
  for pair in 0 2; do
    PFT_PAIR=$pair timeout -k 10 300 python bench.py --grid-nodes $g --steps $st --warmup 50 --no-cpu > $O/g${g}_p$pair.json 2>> $O/err.log || exit 1
    python3 -c "import json;d=json.load(open('$O/g${g}_p$pair.json'));print('g$g pair=$pair', d['value'], d['ms_per_step'], d['roofline']['stages_ms'])"
  done
done
for pair in 0 2; do
  export PFT_PAIR=$pair
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr$pair -o run --output-format csv -- python3 bench.py --grid-nodes 100 --steps 200 --warmup 50 --no-cpu --timing-steps 0 > /dev/null 2>> $O/err.log || exit 1
done
