# Scaler planning sweep (chunk height, segment rows, LDS budget) on one GPU.
# Usage (through gpurun): bash tools/sweep_scale.sh TAG
set -o pipefail
TAG=${1:-sweep}
mkdir -p gpurun_out
out=gpurun_out/sweep_$TAG.txt
: > $out
for cfg in "32 256 40" "64 256 80" "64 540 80" "32 540 40" "32 128 40" "16 256 40" "64 360 64"; do
  set -- $cfg
  PIXPATH_SCALE_CHO_MAX=$1 PIXPATH_SCALE_SEG_ROWS=$2 PIXPATH_SCALE_LDS_KB=$3 \
    timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/sweep_one.json || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sweep_one.json')); print('cho=%s seg=%s lds=%s avpvs_fps=%.0f scale_ms=%.4f siti_ms=%.4f value=%.0f' % (sys.argv[1], sys.argv[2], sys.argv[3], d['avpvs_fps_kernel'], d['roofline']['avg_launch_ms'], 600e3/d['siti_fps_kernel'], d['value']))" $1 $2 $3 | tee -a $out
done
