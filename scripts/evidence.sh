#!/bin/bash
# One GPU-box session producing the round's evidence (TAG=r02 by default; PMC_GIT = the commit, passed in):
#   1. pytest -m gpu, smoke()
#   2. rocprofv3 --kernel-trace --stats of a short bench run, then FETCH_SIZE and WRITE_SIZE in
#      separate --pmc passes (never combined with other tracing) -> profiles/pmc_summary.json
#   3. the default bench line (reads profiles/pmc_summary.json for roofline.traffic), then the
#      secondary numbers of SURVEY 8(d): calc_mode 1 and 2, gl_static, the literal 400^3 cube
# Every GPU step runs under its own time limit; a crash/fault/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r03}
export TAG PMC_DATE=${PMC_DATE:-$(date -u +%F)} PMC_GIT=${PMC_GIT:-unknown}
O=gpurun_out/ev
mkdir -p $O/prof
fatal() { local rc=$1; echo "[$2] exit $rc" | tee -a $O/status.log
  if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then echo "fatal in $2, stopping"; exit "$rc"; fi; }
# PART=1: tests, smoke, traces, PMC passes and the default bench line; PART=2: the other
# workloads; unset: both (a gpurun call is limited to 20 minutes)
PART=${PART:-all}
if [ "$PART" != 2 ] && [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; fatal $? pytest
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; fatal $? smoke
fi
if [ "$PART" != 2 ]; then
ARGS="--steps 20 --warmup 3 --no-cpu --probe 3"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof/trace -o run --output-format csv -- python3 bench.py $ARGS > $O/prof/trace_bench.json 2> $O/prof/trace.err; fatal $? trace
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $O/prof/fetch -o run --output-format csv -- python3 bench.py $ARGS > $O/prof/fetch_bench.json 2> $O/prof/fetch.err; fatal $? fetch
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $O/prof/write -o run --output-format csv -- python3 bench.py $ARGS > $O/prof/write_bench.json 2> $O/prof/write.err; fatal $? write
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $O/prof/valu -o run --output-format csv -- python3 bench.py $ARGS > $O/prof/valu_bench.json 2> $O/prof/valu.err; fatal $? valu
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE -d $O/prof/fp64 -o run --output-format csv -- python3 bench.py $ARGS > $O/prof/fp64_bench.json 2> $O/prof/fp64.err; fatal $? fp64
# L2 hits and misses per kernel (pair 4+5's re-loaded operands)
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum -d $O/prof/tcc -o run --output-format csv -- python3 bench.py $ARGS > $O/prof/tcc_bench.json 2> $O/prof/tcc.err; fatal $? tcc
PB=$(python3 -c "import json;print(json.load(open('$O/prof/trace_bench.json'))['probe_bytes_each_way'])")
python3 scripts/pmc_summary.py $O/prof/trace $O/prof/fetch $O/prof/write 200x200x400 $PB $O/pmc_summary.json $O/prof/valu $O/prof/fp64 > $O/pmc_summary.txt 2>&1; fatal $? pmc_summary
cp $O/pmc_summary.json profiles/pmc_summary.json
timeout -k 10 900 python bench.py > $O/bench_default.json 2> $O/bench_default.err; fatal $? bench_default
# the GPU clock per launch in the driver's configuration, with the bench's clock pre-warm
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE -d $O/prof/clk -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/prof/clk_bench.json 2> $O/prof/clk.err; fatal $? clock
fi
[ "$PART" = 1 ] && { echo done >> $O/status.log; exit 0; }
PFT_PAIR=0 timeout -k 10 300 python bench.py --steps 100 --no-cpu > $O/bench_nopair.json 2>> $O/bench_var.err; fatal $? bench_nopair
timeout -k 10 300 python bench.py --steps 100 --no-cpu --mode 1 > $O/bench_mode1.json 2>> $O/bench_var.err; fatal $? bench_mode1
timeout -k 10 300 python bench.py --steps 100 --no-cpu --mode 2 > $O/bench_mode2.json 2>> $O/bench_var.err; fatal $? bench_mode2
timeout -k 10 300 python bench.py --steps 100 --no-cpu --gl-static > $O/bench_gls.json 2>> $O/bench_var.err; fatal $? bench_gls
timeout -k 10 600 python bench.py --steps 50 --no-cpu --literal-cube > $O/bench_cube64M.json 2>> $O/bench_var.err; fatal $? bench_cube
# the small grids (BASELINE configs[0] and [2]) and the drop-in configuration with a Service_Callback
timeout -k 10 300 python bench.py --steps 2000 --warmup 20 --no-cpu --grid-nodes 100 > $O/bench_g100.json 2>> $O/bench_var.err; fatal $? bench_g100
timeout -k 10 300 python bench.py --steps 400 --no-cpu --grid-nodes 200 > $O/bench_g200.json 2>> $O/bench_var.err; fatal $? bench_g200
timeout -k 10 300 python bench.py --steps 200 --no-cpu --callback > $O/bench_callback.json 2>> $O/bench_var.err; fatal $? bench_callback
timeout -k 10 300 python bench.py --steps 200 --no-cpu --host-boundary > $O/bench_hostb.json 2>> $O/bench_var.err; fatal $? bench_hostb
# per-rank slabs of the N > 1 cube workloads on one GPU, plain and through the N > 1 path of each
# transport with a self-exchanging 1-rank communicator (--self-exchange)
for dom in "400 0.06,0.06,0.015 n8" "318 0.06,0.06,0.03 n4" "252 0.06,0.06,0.06 n2"; do
  set -- $dom
  timeout -k 10 300 python bench.py --steps 100 --no-cpu --grid-nodes $1 --domain $2 > $O/bench_slab_$3.json 2>> $O/bench_var.err; fatal $? slab_$3
  for tr in ipc ipc-ce rccl; do
    timeout -k 10 300 python bench.py --steps 100 --no-cpu --grid-nodes $1 --domain $2 --self-exchange --transport $tr > $O/bench_slab_$3_selfx_$tr.json 2>> $O/bench_var.err; fatal $? slab_$3_selfx_$tr
  done
done
# the driver's own configuration (--steps 20 --warmup 5) three times, and its per-launch kernel trace
# (the clock transient after the warm-up)
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_driver_$r.json 2>> $O/bench_var.err; fatal $? bench_driver
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof/driver -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/prof/driver_bench.json 2> $O/prof/driver.err; fatal $? driver_trace
# bench.py --gpus N rehearsed on this one GPU (ipc ranks) with its decomposition parity check
bash scripts/bench_multi.sh > $O/bench_multi.log 2>&1; fatal $? bench_multi
TRANSPORT=ipc-ce TAG=_ce bash scripts/bench_multi.sh > $O/bench_multi_ce.log 2>&1; fatal $? bench_multi_ce
echo done >> $O/status.log
