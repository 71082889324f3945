#!/bin/bash
# Per-kernel average durations (rocprofv3 --kernel-trace --stats) of the default bench workload on
# every library in $LIBS, for builds whose results are not meant to be right (timing experiments:
# the bench's own timing pass may end early there).  Outputs under gpurun_out/abt/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/abt
mkdir -p $O
for rep in $(seq ${REPS:-1}); do
  for lib in ${LIBS:-lib lib_alt}; do
    PFT_LIB=$PWD/porousfreezethaw_amd/$lib/libpft.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${lib}_r$rep -o run --output-format csv -- python3 bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu --timing-steps 0 $ARGS > $O/${lib}_r$rep.json 2>> $O/err.log || { echo "$lib failed"; exit 1; }
    python3 - $O/${lib}_r$rep/run_kernel_stats.csv $lib <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "merson" in r["Name"]]
print(sys.argv[2].ljust(10), "  ".join(f"{r['Name'].split('(')[0].replace('void ', '')}: {float(r['AverageNs'])/1e3:.1f}us x{r['Calls']}" for r in rows))
PY
  done
done
