# Chunk-height / segment sweep of the scaler plan (measurement only).
# Usage: CFGS="32:256 32:540" bash tools/sweep_cho.sh
set -o pipefail
mkdir -p gpurun_out
for rep in ${REPS:-1}; do
for cfg in ${CFGS:-32:256 24:256 48:256 16:256 24:540 32:540}; do
  c=${cfg%%:*}; s=${cfg##*:}
  PIXPATH_SCALE_CHO_MAX=$c PIXPATH_SCALE_SEG_ROWS=$s timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --pvs-per-rank 8 --no-cpu-baseline --no-pipeline $BARGS > gpurun_out/cho_${c}_${s}.json 2>gpurun_out/cho.err || { tail -3 gpurun_out/cho.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/cho_${c}_${s}.json')); print('rep=$rep cho=$c seg=$s', d['roofline']['avg_launch_ms'])"
done
done
