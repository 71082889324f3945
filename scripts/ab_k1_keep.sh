cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/abk1
for r in 1 2 3; do for lib in lib lib_alt; do
  PFT_LIB=$PWD/porousfreezethaw_amd/$lib/libpft.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/abk1/${lib}_$r.json 2>>gpurun_out/abk1/err.log || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/abk1/${lib}_$r.json'));print('$lib'.ljust(8), d['value'], d['ms_per_step'])"
done; done
