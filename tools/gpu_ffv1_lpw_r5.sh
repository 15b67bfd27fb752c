# FFV1 decoder lanes per wave (measurement build PIXPATH_FFV1_LPW, which sets the
# coder's lanes too: read the decode numbers) with the 63-context records.
# Usage: bash tools/gpu_ffv1_lpw_r5.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for l in 16 24 32 48 64; do
    PIXPATH_FFV1_LPW=$l PIXPATH_LIB=tools/ablate/libpixpath_ablate.so timeout -k 10 200 python -u bench.py --allow-tuning \
        --workload ffv1 --steps 3 --warmup 1 --no-cpu-baseline --ffv1-concurrent 1 > gpurun_out/lpw${l}_${rep}_$TAG.json \
        2>> gpurun_out/lpw_$TAG.err || { tail -3 gpurun_out/lpw_$TAG.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('lpw $l', $rep, 'dec', d['decode']['frames_per_s'], d['decode']['lossless'], 'enc', d['value'])" gpurun_out/lpw${l}_${rep}_$TAG.json
  done
done
