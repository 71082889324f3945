#!/bin/bash
# kernel + memory-copy trace of the 800^3 rank slab with the copy-engine self exchange ($1: output tag;
# env as set by the caller, e.g. PFT_CE_BND=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=$PWD/gpurun_out/cetrace_$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --prewarm-s 0 --no-cpu --no-timing --grid-nodes 400 \
  --domain 0.06,0.06,0.015 --self-exchange --transport ${TR:-ipc-ce} > $OUT/bench.json 2> $OUT/err.log
