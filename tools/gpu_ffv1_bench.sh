# FFV1 encoder: bench lines (4x4 and 8x8 slice grids) + rocprof kernel stats.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --workload ffv1 --steps 3 --warmup 1 > gpurun_out/bench_ffv1_4x4.json 2> gpurun_out/bench_ffv1.err || { tail -5 gpurun_out/bench_ffv1.err; exit 1; }
cat gpurun_out/bench_ffv1_4x4.json
timeout -k 10 200 python -u bench.py --workload ffv1 --steps 3 --warmup 1 --ffv1-slices 8x8 --no-cpu-baseline > gpurun_out/bench_ffv1_8x8.json 2>> gpurun_out/bench_ffv1.err || { tail -5 gpurun_out/bench_ffv1.err; exit 1; }
cat gpurun_out/bench_ffv1_8x8.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_ffv1 -o run -- python3 bench.py --workload ffv1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/kt_ffv1.log 2>&1 || { tail -5 gpurun_out/kt_ffv1.log; exit 1; }
grep -E "ffv1" gpurun_out/kt_ffv1/run_kernel_stats.csv | cut -d, -f1-5
