# Plan geometry sweep (env overrides, no rebuild): config-4 chain chunk height /
# segment rows, config-2 strip segment rows.  Usage: bash tools/gpu_geom_sweep.sh TAG
. tools/ablate_env.sh
set -o pipefail
TAG=${1:-geo}
mkdir -p gpurun_out
export TMPDIR=/tmp
for cho in 16 32; do for seg in 270 540; do
  PIXPATH_SCALE_CHO_MAX=$cho PIXPATH_SCALE_SEG_ROWS=$seg timeout -k 10 120 python -u bench.py $BENCH_TUNE --workload config4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/geo_c4_${cho}_${seg}_$TAG.json 2>> gpurun_out/geo_$TAG.err || { tail -3 gpurun_out/geo_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/geo_c4_${cho}_${seg}_$TAG.json'));c=d['canvas_chain'];print('c4 cho $cho seg $seg', c['avg_launch_ms'], c['frac'])"
done; done
for seg in 270 360 540 1080; do
  PIXPATH_SCALE_SEG_ROWS=$seg timeout -k 10 120 python -u bench.py $BENCH_TUNE --steps 10 --warmup 2 --pvs-total 32 --no-cpu-baseline --no-pipeline --no-siti-file --no-e2e > gpurun_out/geo_c2_${seg}_$TAG.json 2>> gpurun_out/geo_$TAG.err || { tail -3 gpurun_out/geo_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/geo_c2_${seg}_$TAG.json'));print('c2 seg $seg', d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done
