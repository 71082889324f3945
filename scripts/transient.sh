#!/bin/bash
# The driver's bench configuration (--steps 20 --warmup 5) repeated, and one per-launch kernel
# trace of it: shows how the pair kernels' launch times evolve over the first steps after the
# warm-up (VERDICT r02 "What's weak" 3).  Outputs under gpurun_out/tr/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/tr
mkdir -p $O
ARGS=${ARGS:-"--steps 20 --warmup 5 --no-cpu"}
for r in 1 2 3; do
  timeout -k 10 300 python bench.py $ARGS > $O/bench_$r.json 2> $O/bench_$r.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 bench.py $ARGS > $O/trace_bench.json 2> $O/trace.err || exit $?
echo done > $O/status.log
