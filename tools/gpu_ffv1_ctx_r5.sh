# FFV1 context-model study: encode / decode frames/s and bytes per frame of
# pixpath's intra stream with smaller 3-input quantisers (measurement build,
# PIXPATH_FFV1_QBOUNDS = the thresholds; the record describes them, the
# product decoder reads it through its general path), lossless round trip
# checked by the bench line.  Then the product library's FFV1 timing against
# the frames per batch, the reference-shaped stream decode and an e2e trace.
# Usage: bash tools/gpu_ffv1_ctx_r5.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
ABL=tools/ablate/libpixpath_ablate.so
for qb in default 3,8,32 2,6,16,48 4,32 3,24; do
  if [ $qb = default ]; then extra=""; else extra="PIXPATH_FFV1_QBOUNDS=$qb"; fi
  env $extra PIXPATH_LIB=$ABL timeout -k 10 240 python -u bench.py --allow-tuning --workload ffv1 --steps 3 --warmup 1 \
      --no-cpu-baseline --ffv1-concurrent 4 > gpurun_out/ffv1ctx_${qb}_$TAG.json 2>> gpurun_out/ffv1ctx_$TAG.err \
      || { tail -5 gpurun_out/ffv1ctx_$TAG.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['concurrent'];print('$qb', 'enc', d['value'], 'dec', d['decode']['frames_per_s'], d['decode']['lossless'], 'B/frame', d['config']['bytes_per_frame'], 'conc4 enc', c['encode_frames_per_s'], 'dec', c['decode_frames_per_s'], c['lossless'])" gpurun_out/ffv1ctx_${qb}_$TAG.json
done
bash tools/gpu_ffv1_split_r5.sh $TAG
