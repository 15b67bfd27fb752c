# FFV1 iteration: the FFV1 / CLI / config GPU tests, the content probe, the
# bench ffv1 line with rocprof kernel stats, and the e2e AVPVS field.
set -o pipefail
TAG=${1:-r3}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ffv1.py tests/test_gpu_cli.py tests/test_gpu_configs.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_ffv1_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_ffv1_$TAG.log; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_ffv1_$TAG.log | head -20
if [ $rc -gt 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u tools/ffv1_probe.py 600 > gpurun_out/ffv1_probe_$TAG.jsonl 2> gpurun_out/ffv1_probe_$TAG.err || { tail -5 gpurun_out/ffv1_probe_$TAG.err; exit 1; }
cat gpurun_out/ffv1_probe_$TAG.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_ffv1_$TAG -o run -- python3 bench.py --workload ffv1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/kt_ffv1_$TAG.log 2>&1 || { tail -5 gpurun_out/kt_ffv1_$TAG.log; exit 1; }
grep -E "ffv1" gpurun_out/kt_ffv1_$TAG/run_kernel_stats.csv | cut -d, -f1-5
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --pvs-total 8 --no-cpu-baseline --no-pipeline --no-siti-file > gpurun_out/bench_e2e_$TAG.json 2> gpurun_out/bench_e2e_$TAG.err || { tail -5 gpurun_out/bench_e2e_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_e2e_$TAG.json'));print(json.dumps(d.get('e2e_avpvs')))"
