set -o pipefail
mkdir -p gpurun_out
run() { PIXPATH_LIB=$PWD/$2 timeout -k 10 120 python bench.py --workload $1 --steps 8 --warmup 2 --pvs-per-rank 4 --no-cpu-baseline --no-pipeline > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -3 gpurun_out/ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$1 $2', d['roofline']['avg_launch_ms'], d['roofline']['frac'])"; }
B=processing-chain_amd/pixpath/libpixpath.so
for rep in 1 2; do
run config3-8 $B; run config3-8 tools/variant_U8_WIDE_4.so; run config3-8 tools/variant_U8_WIDE_5.so
run config2 $B; run config2 tools/variant_NARROW_4.so
run config3-10 $B
done
