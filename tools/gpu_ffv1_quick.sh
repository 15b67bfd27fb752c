set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ffv1.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pt_ffv1.log 2>&1; rc=$?
tail -2 gpurun_out/pt_ffv1.log
[ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pt_ffv1.log | head; exit $rc; }
for g in 4x4 8x8 16x16; do
timeout -k 10 200 python -u bench.py --workload ffv1 --steps 3 --warmup 1 --ffv1-slices $g --no-cpu-baseline > gpurun_out/bench_ffv1_$g.json 2>> gpurun_out/bench_ffv1.err || { tail -5 gpurun_out/bench_ffv1.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_ffv1_$g.json')); print('$g', d['value'], d['ms_per_step'], d['config']['compression'])"
done
