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
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/meas_$TAG/aux_fetch -o run -- python3 tools/aux_kernels.py --launches 2 > gpurun_out/meas_$TAG/aux_fetch.log 2>&1 || { echo "aux fetch pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/meas_$TAG/aux_write -o run -- python3 tools/aux_kernels.py --launches 2 > gpurun_out/meas_$TAG/aux_write.log 2>&1 || { echo "aux write pass failed"; exit 1; }
python3 tools/aux_pmc.py gpurun_out/meas_$TAG/aux_fetch/run_counter_collection.csv gpurun_out/meas_$TAG/aux_write/run_counter_collection.csv gpurun_out/meas_$TAG/aux_kernels.json 2 gpurun_out/meas_$TAG/aux_pmc.json | grep -E "case|over"
for wl in config3-10 config3-8 config4; do
  timeout -k 10 300 python3 bench.py --workload $wl --no-cpu-baseline > gpurun_out/meas_$TAG/bench_$wl.json 2> gpurun_out/meas_$TAG/bench_$wl.err || { tail -5 gpurun_out/meas_$TAG/bench_$wl.err; exit 1; }
  cut -c1-400 gpurun_out/meas_$TAG/bench_$wl.json
done
