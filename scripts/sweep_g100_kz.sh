cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/sw
for r in 1 2; do
for kz in 0 1 2 3 5; do
  timeout -k 10 120 python bench.py --grid-nodes 100 --steps 2000 --warmup 20 --no-cpu --kz $kz --prewarm-s 0.2 > gpurun_out/sw/kz$kz.json 2>>gpurun_out/sw/err.log || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/sw/kz$kz.json'));print('kz $kz', d['value'], round(d['ms_per_step']*1e3,1), d['roofline']['stages_ms'])"
done
done
