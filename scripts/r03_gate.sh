#!/bin/bash
# f4 gated steps: GPU tests (gate, g100, parity, control flow, ABI), then A/B bench lines at 100^3
# and 200^3 (gate on/off, interleaved), the driver's 400^3 configuration with the clock pre-warm,
# and one kernel trace of the gated 100^3 run.  Outputs under gpurun_out/gt/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/gt
mkdir -p $O
TESTS=${TESTS:-"tests/test_gate_gpu.py tests/test_g100.py tests/test_control_flow.py tests/test_abi_gpu.py tests/test_gpu_parity.py"}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider $TESTS > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for g in 1 0; do
    PFT_GATE_TRACE=1 timeout -k 10 300 python bench.py --grid-nodes 100 --steps 2000 --warmup 20 --no-cpu --gate $g > $O/g100_gate${g}_$r.json 2>> $O/err.log || exit 1
    python3 -c "import json;d=json.load(open('$O/g100_gate${g}_$r.json'));print('g100 gate=$g', d['value'], d['ms_per_step']*1e3, 'us', d['config']['gated_steps'], d['config']['gate_misses'])"
  done
done
for g in 1 0; do
  timeout -k 10 300 python bench.py --grid-nodes 200 --steps 400 --warmup 20 --no-cpu --gate $g > $O/g200_gate$g.json 2>> $O/err.log || exit 1
  python3 -c "import json;d=json.load(open('$O/g200_gate$g.json'));print('g200 gate=$g', d['value'], d['ms_per_step']*1e3, 'us', d['config']['gated_steps'])"
done
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > $O/drv_$r.json 2>> $O/err.log || exit 1
  python3 -c "import json;d=json.load(open('$O/drv_$r.json'));print('driver cfg', d['value'], d['ms_per_step'], d['config']['clock_prewarm'])"
done
PFT_GATE_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 bench.py --grid-nodes 100 --steps 400 --warmup 20 --no-cpu --timing-steps 0 > $O/tr_bench.json 2>> $O/err.log || exit 1
echo done
