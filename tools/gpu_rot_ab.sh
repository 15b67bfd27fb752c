# strip_kernel rotated H-window reads: scaler parity, then same-box A/B vs tools/libvariants/strip_norot.so
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_scale_long.py tests/test_gpu_chain.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pt_rot.log 2>&1; rc=$?
tail -2 gpurun_out/pt_rot.log; grep -E "^(FAILED|ERROR)" gpurun_out/pt_rot.log | head -5
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for lib in processing-chain_amd/pixpath/libpixpath.so tools/libvariants/strip_norot.so; do
  for wl in config3-8 config3-10 config2; do
    PIXPATH_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --workload $wl --steps 6 --warmup 2 --pvs-per-rank 4 --no-cpu-baseline --no-pipeline > gpurun_out/rab.json 2> gpurun_out/rab.err || { tail -3 gpurun_out/rab.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/rab.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$wl', '$lib'.split('/')[-1], r['avg_launch_ms'], r['frac'])"
  done
done
done
