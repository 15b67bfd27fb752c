# Round-6 A/B of strip_kernel library variants (config 2, config 4 chain,
# config 3 8-bit), interleaved, after the scaler GPU tests on the new library.
# usage (through gpurun): bash tools/gpu_r6_ab.sh TAG variant1 [variant2 ...]
#   variant "product" = processing-chain_amd/pixpath/libpixpath.so, else tools/var/libpixpath_<v>.so
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests/test_gpu_scale.py tests/test_gpu_scale_long.py tests/test_gpu_chain.py tests/test_gpu_configs.py tests/test_gpu_ffv1.py tests/test_gpu_ffv1_general.py tests/test_gpu_pack.py}
if [ -z "$NOTEST" ]; then
timeout -k 10 800 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/ab_pytest_$TAG.log 2>&1; rc=$?
tail -2 gpurun_out/ab_pytest_$TAG.log; grep -E "^(FAILED|ERROR)" gpurun_out/ab_pytest_$TAG.log | head
[ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
fi
lib() { if [ $1 = product ]; then echo $PWD/processing-chain_amd/pixpath/libpixpath.so; else echo $PWD/tools/var/libpixpath_$1.so; fi; }
for rep in 1 2; do
  for v in "$@"; do
    PIXPATH_LIB=$(lib $v) timeout -k 10 120 python3 bench.py --allow-tuning --steps 10 --warmup 3 --pvs-total 32 --no-cpu-baseline --no-pipeline --no-siti-file --no-e2e > gpurun_out/ab_${TAG}_c2_$v.json 2> gpurun_out/ab_${TAG}_c2_$v.err || { tail -3 gpurun_out/ab_${TAG}_c2_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab_${TAG}_c2_$v.json'));r=d['roofline'];print('c2 $v', r['avg_launch_ms'], r['frac'], 'siti', d['siti_kernel']['avg_launch_ms'])"
  done
  for wl in config4 config3-8; do
  for v in "$@"; do
    PIXPATH_LIB=$(lib $v) timeout -k 10 120 python3 bench.py --allow-tuning --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline --no-siti-file > gpurun_out/ab_${TAG}_${wl}_$v.json 2> gpurun_out/ab_${TAG}_${wl}_$v.err || { tail -3 gpurun_out/ab_${TAG}_${wl}_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab_${TAG}_${wl}_$v.json'));r=d['roofline'];c=d.get('canvas_chain') or {};print('$wl $v', r['avg_launch_ms'], r['frac'], 'write_gbs', d.get('write_gbs'), 'chain', c.get('avg_launch_ms'), c.get('frac'))"
  done
  done
done
