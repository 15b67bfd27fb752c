# Config-4 chain: FUSE 11 (chroma launch) at a 7-wave register floor (72 VGPRs,
# 2 spilled; libpixpath_c11w7.so) vs the product's 6 (measurement builds),
# alternating, after chain parity of the variant.  Usage: bash tools/gpu_chroma_occ_r5.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
PIXPATH_LIB=tools/ablate/libpixpath_c11w7.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_gpu_chain.py > gpurun_out/c11w7_pytest_$TAG.log 2>&1 || { tail -5 gpurun_out/c11w7_pytest_$TAG.log; exit 1; }
echo "parity (c11w7): $(tail -1 gpurun_out/c11w7_pytest_$TAG.log)"
for rep in 1 2 3; do
  for lib in ablate c11w7; do
    PIXPATH_LIB=tools/ablate/libpixpath_$lib.so timeout -k 10 200 python -u bench.py --allow-tuning \
        --workload config4 --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/c11_${lib}_${rep}_$TAG.json \
        2>> gpurun_out/c11_$TAG.err || { tail -3 gpurun_out/c11_$TAG.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['canvas_chain'];print('$lib', $rep, c['avg_launch_ms'], c['frac'])" gpurun_out/c11_${lib}_${rep}_$TAG.json
  done
done
