#!/bin/bash
# Quick GPU check of a kernel change: the pair-kernel parity tests, then the driver's bench
# configuration 3x and one per-launch kernel trace of it (scripts/transient.sh).  Stops at the
# first failure.  Outputs under gpurun_out/q/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/q
mkdir -p $O
TESTS=${TESTS:-tests/test_pair_gpu.py}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider $TESTS > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
ARGS=${ARGS:-"--steps 20 --warmup 5 --no-cpu"}
for r in 1 2 3; do
  timeout -k 10 300 python bench.py $ARGS > $O/bench_$r.json 2> $O/bench_$r.err || exit $?
  python3 -c "import json;d=json.load(open('$O/bench_$r.json'));print(d['value'],d['ms_per_step'],d['roofline']['stages_ms'])"
done
timeout -k 10 300 python bench.py --steps 200 --no-cpu > $O/bench_200.json 2> $O/bench_200.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench_200.json'));print('200 steps',d['value'],d['ms_per_step'],d['roofline']['stages_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py $ARGS > $O/trace_bench.json 2> $O/trace.err || exit $?
echo done > $O/status.log
# the GPU clock per launch: GRBM_GUI_ACTIVE (busy GPU cycles) over each dispatch's duration
if [ -n "$CLOCK" ]; then
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $O/clk -o run --output-format csv -- python3 bench.py $ARGS > $O/clk_bench.json 2> $O/clk.err || exit $?
fi
