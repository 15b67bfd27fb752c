# FFV1 lanes-per-wave sweep (coder + decoder), FFV1/chain parity tests, the
# config-4 chain line.  Usage (through gpurun): bash tools/gpu_ffv1_lpw.sh TAG
set -o pipefail
TAG=${1:-lpw}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ffv1.py tests/test_gpu_chain.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_lpw_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_lpw_$TAG.log; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_lpw_$TAG.log | head -20
if [ $rc -gt 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
for lpw in ${LPWS:-64 32 16}; do
  PIXPATH_FFV1_LPW=$lpw timeout -k 10 200 python -u bench.py --workload ffv1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ffv1_lpw${lpw}_$TAG.json 2>> gpurun_out/ffv1_lpw_$TAG.err || { tail -5 gpurun_out/ffv1_lpw_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ffv1_lpw${lpw}_$TAG.json'));print('lpw $lpw enc',d['value'],'dec',d['decode']['frames_per_s'],d['decode']['lossless'])"
done
timeout -k 10 200 python -u bench.py --workload config4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_config4_$TAG.json 2>> gpurun_out/ffv1_lpw_$TAG.err || { tail -5 gpurun_out/ffv1_lpw_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_config4_$TAG.json'));print('config4', d['value'], d['roofline'])"
