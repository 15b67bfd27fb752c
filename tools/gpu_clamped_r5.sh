# Config-4 chain: FUSE 9/11 compiled with the clamped V pass alone (FUSE 11 at a
# 7-wave floor) vs the previous state (libpixpath_prev.so: both loop copies, 6
# waves), measurement builds, alternating, after the product's chain and
# config-4 parity.  Usage: bash tools/gpu_clamped_r5.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py \
    -k "chain or config4" tests/test_gpu_configs.py > gpurun_out/clamped_pytest_$TAG.log 2>&1; rc=$?
echo "parity: $(tail -1 gpurun_out/clamped_pytest_$TAG.log)"
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" gpurun_out/clamped_pytest_$TAG.log | head; exit $rc; fi
for rep in 1 2 3; do
  for lib in ablate prev; do
    PIXPATH_LIB=tools/ablate/libpixpath_$lib.so timeout -k 10 200 python -u bench.py --allow-tuning \
        --workload config4 --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/clamped_${lib}_${rep}_$TAG.json \
        2>> gpurun_out/clamped_$TAG.err || { tail -3 gpurun_out/clamped_$TAG.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['canvas_chain'];print('$lib', $rep, c['avg_launch_ms'], c['frac'])" gpurun_out/clamped_${lib}_${rep}_$TAG.json
  done
done
