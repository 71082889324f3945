#!/bin/bash
# Counters of the stage and pair kernels in separate rocprofv3 --pmc passes over a short bench run
# (never combined with other tracing): issue and waits, LDS (bank conflicts), L2 hit/miss, and the
# calibrated HBM bytes (FETCH_SIZE, WRITE_SIZE).  -> gpurun_out/$PMC_OUT/table.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${PMC_OUT:-pmc_pair}
mkdir -p $OUT
ARGS="--steps 10 --warmup 2 --no-cpu --timing-steps 0 $BENCH_ARGS"
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $counters -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.json 2> $OUT/p$i.err
  rc=$?; echo "pass $i ($counters) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done <<'LIST'
SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU
SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE
TCC_HIT_sum TCC_MISS_sum GRBM_COUNT
FETCH_SIZE
WRITE_SIZE
LIST
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, os
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(os.path.join(out, "table.txt"), "w") as fh:
    for k, v in sorted(acc.items()):
        if "merson" not in k and "probe" not in k: continue
        line = k.split("(")[0][:40] + " | " + " ".join(f"{c}={sum(x)/len(x):.6g}" for c, x in sorted(v.items()))
        print(line); fh.write(line + "\n")
PY
