#!/bin/bash
# Round-3 re-entry measurement: f4 (100^3 / 200^3 stage launches vs pair kernels, kernel traces)
# and the GPU clock per launch in the driver's 400^3 configuration (GRBM_GUI_ACTIVE pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
bash scripts/small_grid.sh || exit 1
O=gpurun_out/clk
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $O/clk -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/clk_bench.json 2> $O/clk.err || exit 1
echo done
