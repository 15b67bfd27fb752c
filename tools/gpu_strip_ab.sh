# A/B of two builds of libpixpath (PIXPATH_LIB): headline strip_kernel line and
# the config-4 chain line, alternating, after the scaler/chain GPU tests of the new one.
set -o pipefail
TAG=${1:-ab}
OLD=processing-chain_amd/pixpath/libpixpath_old.so
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_chain.py tests/test_gpu_configs.py tests/test_gpu_pack.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_$TAG.log | head
if [ $rc -gt 1 ]; then exit $rc; fi
for r in 1 2; do
for v in old new; do
if [ $v = old ]; then export PIXPATH_LIB=$OLD; else unset PIXPATH_LIB; fi
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_${v}_$TAG.json 2>> gpurun_out/b_$TAG.err || { tail -3 gpurun_out/b_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/b_${v}_$TAG.json'));r=d['roofline'];print('$v strip', d['value'], r['avg_launch_ms'], r['frac'])"
timeout -k 10 120 python -u bench.py --workload config4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c4_${v}_$TAG.json 2>> gpurun_out/b_$TAG.err || { tail -3 gpurun_out/b_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c4_${v}_$TAG.json'));c=d['canvas_chain'];print('$v c4', c['avg_launch_ms'], c['frac'])"
done
done
