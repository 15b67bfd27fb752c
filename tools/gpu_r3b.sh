# Round-3 status session: every GPU test, the default bench line, the FFV1
# bench line with rocprof kernel stats, the FFV1 content probe.
# Usage (through gpurun): bash tools/gpu_r3b.sh TAG
set -o pipefail
TAG=${1:-r3b}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu_$TAG.log | head -20
if [ $rc -gt 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print('value',d['value'],'frac',d['roofline']['frac'],'ms',d['roofline']['avg_launch_ms'],'siti',d['siti_kernel']['avg_launch_ms'],'e2e',d.get('e2e_avpvs'),'pcie',d.get('pcie_pipeline',{}).get('frames_per_s'),'cpu',d['cpu_baseline']['value'])"
timeout -k 10 200 python -u bench.py --workload ffv1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_ffv1_$TAG.json 2> gpurun_out/bench_ffv1_$TAG.err || { tail -5 gpurun_out/bench_ffv1_$TAG.err; exit 1; }
cat gpurun_out/bench_ffv1_$TAG.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_ffv1_$TAG -o run -- python3 bench.py --workload ffv1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/kt_ffv1_$TAG.log 2>&1 || { tail -5 gpurun_out/kt_ffv1_$TAG.log; exit 1; }
grep -E "ffv1" gpurun_out/kt_ffv1_$TAG/run_kernel_stats.csv | cut -d, -f1-5
timeout -k 10 300 python -u tools/ffv1_probe.py 600 > gpurun_out/ffv1_probe_$TAG.jsonl 2> gpurun_out/ffv1_probe_$TAG.err || { tail -5 gpurun_out/ffv1_probe_$TAG.err; exit 1; }
cat gpurun_out/ffv1_probe_$TAG.jsonl
