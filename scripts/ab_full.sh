#!/bin/bash
# Full GPU parity suite on lib/, then the lib vs lib_alt A/B sweep (scripts/ab_sweep.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ge 124 ] && exit $rc
[ $rc -ne 0 ] && exit $rc
bash scripts/ab_sweep.sh
