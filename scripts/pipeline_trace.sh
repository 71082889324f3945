#!/bin/bash
# Kernel trace of the N > 1 stage pipeline, rehearsed on one GPU (1-rank RCCL self-exchange) on the
# 400x400x100 slab of one 800^3 8-way rank, plus the small-grid and host-boundary bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/ptrace; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-timing --grid-nodes 400 --domain 0.06,0.06,0.015 --self-exchange > $O/selfx_trace_bench.json 2> $O/tr.err || exit 1
timeout -k 10 200 python bench.py --steps 200 --no-cpu --grid-nodes 100 > $O/g100.json 2>>$O/err.log || exit 1
timeout -k 10 200 python bench.py --steps 200 --no-cpu --grid-nodes 200 > $O/g200.json 2>>$O/err.log || exit 1
timeout -k 10 300 python bench.py --steps 200 --no-cpu --host-boundary > $O/hostb.json 2>>$O/err.log || exit 1
echo ok
