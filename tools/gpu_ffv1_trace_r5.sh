# FFV1 GPU tests, then a kernel trace of bench --workload ffv1 (per-kernel times).
# Usage: bash tools/gpu_ffv1_trace_r5.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_r5.sh $TAG tests:ffv1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ffv1_trace_$TAG -o run -- \
    python3 -u bench.py --workload ffv1 --steps 3 --warmup 1 --no-cpu-baseline --ffv1-concurrent 1 \
    > gpurun_out/ffv1_trace_$TAG.json 2> gpurun_out/ffv1_trace_$TAG.err || { tail -5 gpurun_out/ffv1_trace_$TAG.err; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('enc', d['value'], 'dec', d['decode']['frames_per_s'])" gpurun_out/ffv1_trace_$TAG.json
grep -E "ffv1" gpurun_out/ffv1_trace_$TAG/run_kernel_stats.csv | cut -d, -f1-4
