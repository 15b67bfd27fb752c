# A/B of the headline strip kernel (config 2) across library variants, interleaved.
set -o pipefail
export TMPDIR=/tmp
for rep in 1 2; do
for v in product g8 noprio seg1080 cho48; do
  if [ $v = product ]; then lib=$PWD/processing-chain_amd/pixpath/libpixpath.so; else lib=$PWD/tools/ablate/libpixpath_$v.so; fi
  PIXPATH_LIB=$lib timeout -k 10 120 python3 bench.py --allow-tuning --steps 10 --warmup 3 --pvs-total 32 --no-cpu-baseline --no-pipeline --no-siti-file --no-e2e > gpurun_out/sv_$v.json 2> gpurun_out/sv_$v.err || { tail -3 gpurun_out/sv_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sv_$v.json'));r=d['roofline'];print('$v', r['avg_launch_ms'], r['frac'], 'siti', d['siti_kernel']['avg_launch_ms'])"
done
done
