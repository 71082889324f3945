#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
timeout -k 10 300 python bench.py --steps 60 --warmup 5 --no-cpu --kz 8 > gpurun_out/diag/normal.json 2>gpurun_out/diag/err.log || exit $?
PFT_LIB=$PWD/porousfreezethaw_amd/lib_ablate/libpft.so timeout -k 10 300 python bench.py --steps 60 --warmup 5 --no-cpu --kz 8 > gpurun_out/diag/ablate.json 2>>gpurun_out/diag/err.log || exit $?
timeout -k 10 120 rocprofv3 -L > gpurun_out/diag/counters.txt 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/diag/sq -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu --kz 8 > gpurun_out/diag/sq.json 2> gpurun_out/diag/sq.err
echo "sq rc=$?"
python3 - <<'PY'
import json
for n in ("normal","ablate"):
    d=json.load(open(f"gpurun_out/diag/{n}.json")); print(n, d["value"], d["roofline"]["stages_ms"])
PY
