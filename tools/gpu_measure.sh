# Measurement pass: non-scaler kernel rooflines (HIP events + rocprof), config 3/4 bench lines.
# Usage (through gpurun): bash tools/gpu_measure.sh TAG
set -o pipefail
TAG=${1:-m}
export TMPDIR=/tmp
mkdir -p gpurun_out/meas_$TAG
timeout -k 10 300 python3 tools/aux_kernels.py --out gpurun_out/meas_$TAG/aux_kernels.json > gpurun_out/meas_$TAG/aux.log 2>&1 || { tail -5 gpurun_out/meas_$TAG/aux.log; exit 1; }
cat gpurun_out/meas_$TAG/aux.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/meas_$TAG/aux_kt -o run -- python3 tools/aux_kernels.py --launches 3 > gpurun_out/meas_$TAG/aux_kt.log 2>&1 || { echo "aux rocprof failed"; exit 1; }
grep -E "pp::" gpurun_out/meas_$TAG/aux_kt/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-140
for wl in config3-10 config3-8 config4; do
  timeout -k 10 300 python3 bench.py --workload $wl --no-cpu-baseline > gpurun_out/meas_$TAG/bench_$wl.json 2> gpurun_out/meas_$TAG/bench_$wl.err || { tail -5 gpurun_out/meas_$TAG/bench_$wl.err; exit 1; }
  cut -c1-400 gpurun_out/meas_$TAG/bench_$wl.json
done
