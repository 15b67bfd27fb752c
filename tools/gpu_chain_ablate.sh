# config-4 chain kernel ablation (PIXPATH_SCALE_DEBUG bits: 1 no V-pass stores, 2 no staging
# loads, 4 no H pass, 8 no barriers; timing only) and chunk height 24.
. tools/ablate_env.sh
set -o pipefail
TAG=${1:-cab}
mkdir -p gpurun_out
export TMPDIR=/tmp
for dbg in ${DBGS:-0 1 2 4 8 6}; do
  PIXPATH_SCALE_DEBUG=$dbg timeout -k 10 120 python -u bench.py $BENCH_TUNE --workload config4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/cab_${dbg}_$TAG.json 2>> gpurun_out/cab_$TAG.err || { tail -3 gpurun_out/cab_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/cab_${dbg}_$TAG.json'));c=d['canvas_chain'];print('debug $dbg', c['avg_launch_ms'])"
done
PIXPATH_SCALE_CHO_MAX=24 timeout -k 10 120 python -u bench.py $BENCH_TUNE --workload config4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/cab_cho24_$TAG.json 2>> gpurun_out/cab_$TAG.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/cab_cho24_$TAG.json'));c=d['canvas_chain'];print('cho 24', c['avg_launch_ms'])"
