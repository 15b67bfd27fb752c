# Round 6: config-4 chain knob sweep on the measurement build (tools/ablate).  usage: bash tools/gpu_r6_chain_sweep.sh TAG
set -o pipefail
TAG=${1:-sw}
mkdir -p gpurun_out
export TMPDIR=/tmp
ABL=$PWD/tools/var/libpixpath_abl.so
one() {  # label env...
  local l=$1; shift
  env "$@" PIXPATH_LIB=$ABL timeout -k 10 120 python3 bench.py --allow-tuning --workload config4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sw_${TAG}_$l.json 2> gpurun_out/sw_${TAG}_$l.err || { tail -3 gpurun_out/sw_${TAG}_$l.err; return 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sw_${TAG}_$l.json'));c=d['canvas_chain'];print('$l', c['avg_launch_ms'], c['frac'])"
}
for rep in 1 2 3; do
one base X=1 || exit 1
if [ -n "$COMBOS" ]; then
one s3l40 PIXPATH_CHAIN_SEG2=3 PIXPATH_CHAIN_LUMA_CHO=40 || exit 1
one s2l40 PIXPATH_CHAIN_SEG2=2 PIXPATH_CHAIN_LUMA_CHO=40 || exit 1
one l48 PIXPATH_CHAIN_LUMA_CHO=48 || exit 1
one l40r270 PIXPATH_CHAIN_LUMA_CHO=40 PIXPATH_SCALE_SEG_ROWS=270 || exit 1
one s3l40r270 PIXPATH_CHAIN_SEG2=3 PIXPATH_CHAIN_LUMA_CHO=40 PIXPATH_SCALE_SEG_ROWS=270 || exit 1
else
one seg2_2 PIXPATH_CHAIN_SEG2=2 || exit 1
one seg2_3 PIXPATH_CHAIN_SEG2=3 || exit 1
one seg2_6 PIXPATH_CHAIN_SEG2=6 || exit 1
one lcho24 PIXPATH_CHAIN_LUMA_CHO=24 || exit 1
one lcho40 PIXPATH_CHAIN_LUMA_CHO=40 || exit 1
one overlap PIXPATH_CHAIN_OVERLAP=1 || exit 1
one segrows270 PIXPATH_SCALE_SEG_ROWS=270 || exit 1
one segrows1080 PIXPATH_SCALE_SEG_ROWS=1080 || exit 1
fi
done
