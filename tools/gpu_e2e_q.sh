set -o pipefail
TAG=${1:-e2e}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ffv1.py tests/test_gpu_cli.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_$TAG.log | head
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --pvs-total 8 --no-cpu-baseline --no-pipeline --no-siti-file > gpurun_out/bench_e2e_$TAG.json 2> gpurun_out/bench_e2e_$TAG.err || { tail -5 gpurun_out/bench_e2e_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_e2e_$TAG.json'));print(json.dumps(d.get('e2e_avpvs'))[:300])"
timeout -k 10 200 python -u bench.py --workload ffv1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ffv1_$TAG.json 2>> gpurun_out/bench_e2e_$TAG.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/ffv1_$TAG.json'));print('enc',d['value'],'dec',d['decode']['frames_per_s'])"
