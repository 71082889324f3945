#!/bin/bash
# rocprofv3 evidence for the bench kernels: kernel trace + stats, then FETCH_SIZE and WRITE_SIZE
# in separate --pmc passes (never combined with other tracing, per the pool's rules).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
ARGS="--steps ${PROF_STEPS:-20} --warmup 3 --no-cpu --probe 3 ${BENCH_ARGS}"
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof/trace_bench.json 2> gpurun_out/prof/trace.err
rc=$?; echo "trace rc=$rc"; fatal $rc && exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof/fetch_bench.json 2> gpurun_out/prof/fetch.err
rc=$?; echo "fetch rc=$rc"; fatal $rc && exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof/write_bench.json 2> gpurun_out/prof/write.err
rc=$?; echo "write rc=$rc"; fatal $rc && exit $rc
PB=$(python3 -c "import json;print(json.load(open('gpurun_out/prof/trace_bench.json'))['probe_bytes_each_way'])")
python3 scripts/pmc_summary.py gpurun_out/prof/trace gpurun_out/prof/fetch gpurun_out/prof/write ${GRID:-400} $PB gpurun_out/prof/pmc_summary.json
