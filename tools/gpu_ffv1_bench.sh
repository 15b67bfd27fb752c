# FFV1 encoder: bench lines (8x8 and 16x16 slice grids) + rocprof kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3}
timeout -k 10 200 python -u bench.py --workload ffv1 --steps 3 --warmup 1 > gpurun_out/bench_ffv1_8x8_$TAG.json 2> gpurun_out/bench_ffv1_$TAG.err || { tail -5 gpurun_out/bench_ffv1_$TAG.err; exit 1; }
cat gpurun_out/bench_ffv1_8x8_$TAG.json
timeout -k 10 200 python -u bench.py --workload ffv1 --steps 3 --warmup 1 --ffv1-slices 16x16 --no-cpu-baseline > gpurun_out/bench_ffv1_16x16_$TAG.json 2>> gpurun_out/bench_ffv1_$TAG.err || { tail -5 gpurun_out/bench_ffv1_$TAG.err; exit 1; }
cat gpurun_out/bench_ffv1_16x16_$TAG.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_ffv1_$TAG -o run -- python3 bench.py --workload ffv1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/kt_ffv1_$TAG.log 2>&1 || { tail -5 gpurun_out/kt_ffv1_$TAG.log; exit 1; }
grep -E "ffv1" gpurun_out/kt_ffv1_$TAG/run_kernel_stats.csv | cut -d, -f1-5
