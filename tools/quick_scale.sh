# Scaler iteration loop (through gpurun): scale parity tests, bench, kernel trace.
# Usage: bash tools/quick_scale.sh TAG
set -o pipefail
TAG=${1:-q}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_scale_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/pt_scale_$TAG.log
grep -E "^FAILED|Error" gpurun_out/pt_scale_$TAG.log | head -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && cat gpurun_out/bench_$TAG.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt_$TAG -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_kt_$TAG.log 2>&1 &&
cut -c1-150 gpurun_out/prof_kt_$TAG/run_kernel_stats.csv
