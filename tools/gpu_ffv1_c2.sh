set -o pipefail
TAG=${1:-c2}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ffv1.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_$TAG.log; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_$TAG.log | head -5
if [ $rc -gt 1 ]; then exit $rc; fi
for g in 8x8 16x16; do
  timeout -k 10 300 python -u bench.py --workload ffv1 --ffv1-slices $g --ffv1-concurrent 4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ffv1c_${g}_$TAG.json 2>> gpurun_out/ffv1c_$TAG.err || { tail -5 gpurun_out/ffv1c_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ffv1c_${g}_$TAG.json'));c=d['concurrent'];print('$g single enc',d['value'],'dec',d['decode']['frames_per_s'],'| K=4 enc',c['encode_frames_per_s'],'dec',c['decode_frames_per_s'],c['lossless'])"
done
