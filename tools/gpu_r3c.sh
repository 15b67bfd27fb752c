# Round-3 iteration: FFV1 / CLI / config GPU tests, the default bench line
# (incl. e2e_avpvs), FFV1 8x8 + 16x16 lines with kernel stats.
set -o pipefail
TAG=${1:-r3c}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ffv1.py tests/test_gpu_cli.py tests/test_gpu_configs.py tests/test_gpu_chain.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_$TAG.log | head -20
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print('value',d['value'],'frac',d['roofline']['frac'],'ms',d['roofline']['avg_launch_ms'],'siti',d['siti_kernel']['avg_launch_ms'],'pcie',d.get('pcie_pipeline',{}).get('frames_per_s'),'cpu',d['cpu_baseline']['value']); print(json.dumps(d.get('e2e_avpvs')))"
for g in 8x8 16x16; do
  timeout -k 10 200 python -u bench.py --workload ffv1 --ffv1-slices $g --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ffv1_${g}_$TAG.json 2>> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ffv1_${g}_$TAG.json'));print('$g enc',d['value'],'dec',d['decode']['frames_per_s'],d['decode']['lossless'],'ratio',d['config']['compression'])"
done
