# Config-4 chain: segment rows of the plans (PIXPATH_SCALE_SEG_ROWS, measurement
# build: the luma launch's 540-row segments make a long last round), alternating.
# Usage: bash tools/gpu_luma_seg_r5.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
PIXPATH_SCALE_SEG_ROWS=272 PIXPATH_LIB=tools/ablate/libpixpath_ablate.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_gpu_chain.py > gpurun_out/seg_pytest_$TAG.log 2>&1 || { tail -5 gpurun_out/seg_pytest_$TAG.log; exit 1; }
echo "parity (seg 272): $(tail -1 gpurun_out/seg_pytest_$TAG.log)"
for rep in 1 2; do
  for seg in default 360 272 216 136; do
    if [ $seg = default ]; then x=""; else x="PIXPATH_SCALE_SEG_ROWS=$seg"; fi
    env $x PIXPATH_LIB=tools/ablate/libpixpath_ablate.so timeout -k 10 200 python -u bench.py --allow-tuning \
        --workload config4 --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/seg_${seg}_${rep}_$TAG.json \
        2>> gpurun_out/seg_$TAG.err || { tail -3 gpurun_out/seg_$TAG.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['canvas_chain'];print('seg $seg', $rep, c['avg_launch_ms'], c['frac'])" gpurun_out/seg_${seg}_${rep}_$TAG.json
  done
done
