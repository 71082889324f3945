#!/bin/bash
# Round 4, small slabs: optional GPU tests ($TESTS), then 100^3 / 200^3 bench lines with the stage
# launches (PFT_PAIR=0) and the pair kernels forced (PFT_PAIR=2), and one kernel trace of each with
# its per-step timeline (step_timeline.py).  Outputs under gpurun_out/$SG_OUT (default sg4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${SG_OUT:-sg4}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS > $O/pytest.log 2>&1
  rc=$?; tail -5 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for g in ${GRIDS:-100 200}; do
  st=$([ $g = 100 ] && echo 2000 || echo 400)
  for pair in ${PAIRS:-0 2}; do
    PFT_PAIR=$pair timeout -k 10 300 python bench.py --grid-nodes $g --steps $st --warmup 50 --no-cpu > $O/g${g}_p$pair.json 2>> $O/err.log || exit 1
    python3 -c "import json;d=json.load(open('$O/g${g}_p$pair.json'));print('g$g pair=$pair', d['value'], d['ms_per_step'], d['roofline']['stages_ms'])"
  done
done
[ -n "$NOTRACE" ] && exit 0
for g in ${GRIDS:-100 200}; do
  for pair in ${PAIRS:-0 2}; do
    PFT_PAIR=$pair timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr${g}_$pair -o run --output-format csv -- python3 bench.py --grid-nodes $g --steps 200 --warmup 50 --no-cpu --timing-steps 0 > /dev/null 2>> $O/err.log || exit 1
    f=$(find $O/tr${g}_$pair -name '*kernel_trace.csv' | head -1)
    echo "== g$g pair=$pair" | tee -a $O/timeline.txt
    python3 scripts/step_timeline.py $f 100 | tee -a $O/timeline.txt
  done
done
