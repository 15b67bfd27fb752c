set -o pipefail
mkdir -p gpurun_out
for wl in config3-10 config3-8 config4; do
  timeout -k 10 200 python -u bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/bench_${wl}_v5.json 2> gpurun_out/bench_$wl.err || { tail -3 gpurun_out/bench_$wl.err; exit 1; }
  cut -c1-300 gpurun_out/bench_${wl}_v5.json
done
