#!/bin/bash
# pair-kernel GPU tests on the default build, then an interleaved A/B of $LIBS (scripts/ab_libs.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab${TAG}
timeout -k 10 600 python -u -m pytest tests/test_pair_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab${TAG}/pytest_pair.log 2>&1 || exit $?
bash scripts/ab_libs.sh > gpurun_out/ab${TAG}/ab.txt 2>&1
