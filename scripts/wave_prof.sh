cd $GRAFT_REPO_ROOT || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/wprof
for w in 0 32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/wprof/w$w -o run --output-format csv -- python3 bench.py --steps 40 --warmup 3 --no-cpu --no-timing --wave $w > gpurun_out/wprof/b$w.json 2> gpurun_out/wprof/e$w.log || { echo "prof $w failed"; exit 1; }
done
echo ok
