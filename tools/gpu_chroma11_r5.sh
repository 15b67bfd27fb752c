# Config-4 chain: the chroma launch on its own FUSE 11 instance (product) vs the
# FUSE 10 chain instance (PIXPATH_CHAIN_NO_CHROMA11, measurement build),
# alternating, after the chain parity tests.  Usage: bash tools/gpu_chroma11_r5.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py \
    -k "chain or config4" tests/test_gpu_configs.py > gpurun_out/chroma11_pytest_$TAG.log 2>&1; rc=$?
echo "parity: $(tail -1 gpurun_out/chroma11_pytest_$TAG.log)"
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" gpurun_out/chroma11_pytest_$TAG.log | head; exit $rc; fi
for rep in 1 2 3; do
  for m in chroma11 fuse10; do
    if [ $m = fuse10 ]; then x="PIXPATH_CHAIN_NO_CHROMA11=1"; else x=""; fi
    env $x PIXPATH_LIB=tools/ablate/libpixpath_ablate.so timeout -k 10 200 python -u bench.py --allow-tuning --workload config4 \
        --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/chroma11_${m}_${rep}_$TAG.json 2>> gpurun_out/chroma11_$TAG.err \
        || { tail -3 gpurun_out/chroma11_$TAG.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['canvas_chain'];print('$m', $rep, c['avg_launch_ms'], c['frac'])" gpurun_out/chroma11_${m}_${rep}_$TAG.json
  done
done
