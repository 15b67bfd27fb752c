. tools/ablate_env.sh
set -o pipefail
TAG=${1:-m}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_ffv1_conc.sh $TAG || exit 1
for lc in 0 32; do
  if [ $lc = 0 ]; then unset PIXPATH_CHAIN_LUMA_CHO; else export PIXPATH_CHAIN_LUMA_CHO=$lc; fi
  timeout -k 10 120 python -u bench.py $BENCH_TUNE --workload config4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c4lc_${lc}_$TAG.json 2>> gpurun_out/c4lc_$TAG.err || { tail -3 gpurun_out/c4lc_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/c4lc_${lc}_$TAG.json'));c=d['canvas_chain'];print('chain luma cho $lc', c['avg_launch_ms'], c['frac'])"
done
