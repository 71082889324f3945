cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/kz
for kz in 0 1 2 3 4 6; do
  PFT_PAIR=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/kz/k$kz -o run --output-format csv -- python3 bench.py --grid-nodes 100 --steps 400 --warmup 20 --no-cpu --timing-steps 0 --kz $kz > gpurun_out/kz/k$kz.json 2>>gpurun_out/kz/err.log || exit 1
  python3 - gpurun_out/kz/k$kz/run_kernel_stats.csv $kz <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "merson" in r["Name"]]
print("kz", sys.argv[2], "  ".join(f"{r['Name'].split('(')[0].replace('void ', '')}: {float(r['AverageNs'])/1e3:.1f}us" for r in rows))
PY
done
