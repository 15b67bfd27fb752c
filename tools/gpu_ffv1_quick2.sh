# FFV1 iteration: parity tests, 8x8 and 16x16 encode/decode lines, code-kernel counters.
set -o pipefail
TAG=${1:-q}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ffv1.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_ffv1q_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_ffv1q_$TAG.log; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_ffv1q_$TAG.log | head -20
if [ $rc -gt 1 ]; then exit $rc; fi
for g in 8x8 16x16; do
  timeout -k 10 200 python -u bench.py --workload ffv1 --ffv1-slices $g --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ffv1_${g}_$TAG.json 2>> gpurun_out/ffv1q_$TAG.err || { tail -5 gpurun_out/ffv1q_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ffv1_${g}_$TAG.json'));print('$g enc',d['value'],'dec',d['decode']['frames_per_s'],d['decode']['lossless'],'ratio',d['config']['compression'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_ffv1_$TAG -o run -- python3 bench.py --workload ffv1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/kt_ffv1_$TAG.log 2>&1 || { tail -5 gpurun_out/kt_ffv1_$TAG.log; exit 1; }
grep -E "ffv1" gpurun_out/kt_ffv1_$TAG/run_kernel_stats.csv | cut -d, -f1-4
