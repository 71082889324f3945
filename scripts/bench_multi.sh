#!/bin/bash
# bench.py --gpus N rehearsed on ONE GPU: N ranks over the ipc transport (RCCL refuses two ranks on
# one GPU), each with its weak-scaling slab, then the decomposition-invariance check (rank 0's
# single-slab re-run).  Then the same with one rank's digest perturbed by one ulp
# (PFT_BENCH_PARITY_PERTURB=1): the run must fail.  Outputs under gpurun_out/bm$TAG/; $TRANSPORT
# selects the transport (default auto).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/bm${TAG}
mkdir -p $O
port=29511
for n in ${NS:-2 4}; do
  port=$((port+1))
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --steps 20 --warmup 5 --transport ${TRANSPORT:-auto} > $O/n$n.json 2> $O/n$n.err || { echo "n=$n failed"; tail -20 $O/n$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/n$n.json'));print('n=$n', d['value'], d['ms_per_step'], d['config']['transport'], d['parity'])"
done
port=$((port+1))
PFT_BENCH_PARITY_PERTURB=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --steps 20 --warmup 5 --transport ${TRANSPORT:-auto} > $O/perturb.json 2> $O/perturb.err
rc=$?
echo "perturbed run exit status $rc (must be nonzero)"
python3 -c "import json;d=json.load(open('$O/perturb.json'));print('perturbed parity', d['parity'])"
[ $rc -ne 0 ]
