cd $GRAFT_REPO_ROOT || exit 1
mkdir -p gpurun_out/wave
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "wavefront" -p no:cacheprovider > gpurun_out/wave/pytest.log 2>&1 || { tail -30 gpurun_out/wave/pytest.log; exit 1; }
tail -3 gpurun_out/wave/pytest.log
for w in 0 64 48 32 24 16 0 32; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 5 --no-cpu --no-timing --wave $w > gpurun_out/wave/b$w.json 2>>gpurun_out/wave/err.log || { echo "bench $w failed"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/wave/b$w.json'));print('wave', $w, d['value'], d['ms_per_step'])"
done
