set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_scale_long.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pt_c3.log 2>&1; rc=$?
tail -1 gpurun_out/pt_c3.log
[ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR)" gpurun_out/pt_c3.log | head; exit $rc; }
for wl in config3-10 config3-8 config2; do
  for pf in 6 3; do
    lib=processing-chain_amd/pixpath/libpixpath.so
    [ $pf = 3 ] && lib=tools/variant_pf3.so
    PIXPATH_LIB=$PWD/$lib timeout -k 10 120 python bench.py --workload $wl --steps 8 --warmup 2 --pvs-per-rank 4 --no-cpu-baseline --no-pipeline > gpurun_out/c3.json 2> gpurun_out/c3.err || { tail -3 gpurun_out/c3.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/c3.json')); print('$wl pf=$pf', d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
  done
done
