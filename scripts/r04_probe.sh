#!/bin/bash
# Round-4 re-entry: the small-slab step structure probe (kernel boundary vs grid barrier vs host
# round trip, scripts/probes/step_probe.hip) and the round-3 kernel's SQ/LDS/L2 counter passes for
# the pair kernels at 400^3 (pmc_pair.sh).  Outputs under gpurun_out/r04p/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 120 ./scripts/probes/step_probe > $O/step_probe.txt 2>&1; rc=$?
cat $O/step_probe.txt
[ $rc -ne 0 ] && exit $rc
PMC_OUT=r04p/pmc timeout -k 10 600 bash scripts/pmc_pair.sh
