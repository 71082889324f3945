#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/fault/timeout (exit >= 124 or 134/139) ends
# the script immediately.  Test failures (pytest exit 1) do not stop the measurement steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_if_fatal() { rc=$1; what=$2; echo "[$what] exit $rc" | tee -a gpurun_out/status.log
  if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then echo "fatal in $what, stopping"; exit "$rc"; fi; }
rocm-smi --showproductname > gpurun_out/rocm_smi.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
stop_if_fatal $? pytest_gpu
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
stop_if_fatal $? smoke
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-100} --warmup 10 > gpurun_out/bench.json 2> gpurun_out/bench.err
stop_if_fatal $? bench
