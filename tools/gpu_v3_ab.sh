set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
for lib in processing-chain_amd/pixpath/libpixpath.so tools/variant_v3.so; do
  PIXPATH_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --pvs-per-rank 8 --no-cpu-baseline --no-pipeline > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -3 gpurun_out/ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$lib', d['roofline']['avg_launch_ms'], d['siti_kernel']['avg_launch_ms'], d['value'])"
done
done
