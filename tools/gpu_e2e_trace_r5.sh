# Kernel trace of the e2e_avpvs line: per-kernel durations of the encodes
# inside the end-to-end run (host frames -> scale -> FFV1 -> AVI) against the
# same kernels in bench --workload ffv1.
# Usage: bash tools/gpu_e2e_trace_r5.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/e2e_trace_$TAG -o run -- \
    python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pipeline --no-siti-file \
    > gpurun_out/e2e_trace_$TAG.json 2> gpurun_out/e2e_trace_$TAG.err || { tail -5 gpurun_out/e2e_trace_$TAG.err; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));e=d['e2e_avpvs'];print('e2e', e['frames_per_s'], e['single_pvs']['frames_per_s'], e['single_pvs']['stages']['encode_s'], e['stages']['encode_s'])" gpurun_out/e2e_trace_$TAG.json
f=$(find gpurun_out/e2e_trace_$TAG -name '*kernel_stats.csv' | head -1)
if [ -n "$f" ]; then grep -E "ffv1|strip|Name" "$f" | cut -d, -f1-8; fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ffv1_trace_$TAG -o run -- \
    python3 -u bench.py --workload ffv1 --steps 3 --warmup 1 --no-cpu-baseline --ffv1-concurrent 1 \
    > gpurun_out/ffv1_trace_$TAG.json 2>> gpurun_out/e2e_trace_$TAG.err || { tail -5 gpurun_out/e2e_trace_$TAG.err; exit 1; }
f=$(find gpurun_out/ffv1_trace_$TAG -name '*kernel_stats.csv' | head -1)
if [ -n "$f" ]; then grep -E "ffv1|Name" "$f" | cut -d, -f1-8; fi
