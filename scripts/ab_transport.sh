#!/bin/bash
# Per-rank rehearsal of the N > 1 path on one GPU: each rank slab of the cube workloads plain,
# then through the ipc transport (put kernel + flag waits per stage) and the rccl pipeline, both
# exchanging with themselves (--self-exchange); two interleaved rounds.  Output: one JSON line per
# run in gpurun_out/abx/runs.jsonl ("tag" added).  Every GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/abx
mkdir -p $O
run() { local tag=$1; shift   # (an environment assignment before `run` reaches bench.py)
  timeout -k 10 300 python bench.py --no-cpu --steps ${STEPS:-100} "$@" > $O/one.json 2>> $O/err.log || { echo "[$tag] failed $?"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/one.json')); d['tag']='$tag'; print(json.dumps(d))" >> $O/runs.jsonl
  python3 -c "import json; d=json.load(open('$O/one.json')); print('$tag', d['value'], d['ms_per_step'])"
}
for round in 1 2; do
  for dom in "400 0.06,0.06,0.015 n8" "318 0.06,0.06,0.03 n4" "252 0.06,0.06,0.06 n2" "400 0.03,0.03,0.06 n1"; do
    set -- $dom
    run "$3_plain_r$round" --grid-nodes $1 --domain $2
    run "$3_ipc_r$round" --grid-nodes $1 --domain $2 --self-exchange --transport ipc
    run "$3_rccl_r$round" --grid-nodes $1 --domain $2 --self-exchange --transport rccl
  done
  run "n1_callback_r$round" --callback
done
