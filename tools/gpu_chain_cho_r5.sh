# Config-4 chain: chroma chunk height 16 (product) / 24 / 32 with the row-pair
# second stage (measurement builds: PIXPATH_CHAIN_CHO), same box, alternating,
# plus chain parity of each variant.  Usage: bash tools/gpu_chain_cho_r5.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in cho24 cho32; do
  PIXPATH_LIB=tools/ablate/libpixpath_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      tests/test_gpu_chain.py > gpurun_out/chain_${v}_pytest_$TAG.log 2>&1; rc=$?
  echo "$v parity: $(tail -1 gpurun_out/chain_${v}_pytest_$TAG.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for rep in 1 2; do
  for v in ablate cho24 cho32; do
    PIXPATH_LIB=tools/ablate/libpixpath_$v.so timeout -k 10 200 python -u bench.py --allow-tuning --workload config4 \
        --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/chain_${v}_${rep}_$TAG.json 2>> gpurun_out/chain_$TAG.err \
        || { tail -3 gpurun_out/chain_$TAG.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['canvas_chain'];print('$v', $rep, c['avg_launch_ms'], c['frac'])" gpurun_out/chain_${v}_${rep}_$TAG.json
  done
done
