#!/bin/bash
# ipc halos direct into the neighbours' ghost planes vs staged through the receive buffer
# (PFT_IPC_STAGED=1, what a neighbour on another GPU gets), on the 800^3 8-way rank slab through
# the N > 1 path (--self-exchange), interleaved.  Outputs under gpurun_out/stg/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/stg
mkdir -p $O
for r in 1 2; do
  for st in 0 1; do
    PFT_IPC_STAGED=$st timeout -k 10 300 python bench.py --steps 100 --no-cpu --grid-nodes 400 --domain 0.06,0.06,0.015 --self-exchange --transport ipc > $O/n8_staged${st}_$r.json 2>> $O/err.log || exit 1
    python3 -c "import json;d=json.load(open('$O/n8_staged${st}_$r.json'));print('staged=$st', d['value'], d['ms_per_step'], d['roofline']['stages_ms'])"
  done
done
