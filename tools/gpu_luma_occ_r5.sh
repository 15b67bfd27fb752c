# Config-4 chain luma launch occupancy: FUSE 9 wave floor 6 (measurement build)
# vs 7 (libpixpath_l9w7.so) x the luma plan's chunk height (PIXPATH_CHAIN_LUMA_CHO:
# LDS 23.9 KB at 32 rows allows 6 workgroups per CU, shorter chunks 7).
# Usage: bash tools/gpu_luma_occ_r5.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
PIXPATH_CHAIN_LUMA_CHO=24 PIXPATH_LIB=tools/ablate/libpixpath_l9w7.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests/test_gpu_chain.py > gpurun_out/occ_pytest_$TAG.log 2>&1 || { tail -5 gpurun_out/occ_pytest_$TAG.log; exit 1; }
echo "parity (w7, luma cho 24): $(tail -1 gpurun_out/occ_pytest_$TAG.log)"
for rep in 1 2; do
  for lib in ablate l9w7; do
    for cho in 32 28 24; do
      PIXPATH_CHAIN_LUMA_CHO=$cho PIXPATH_LIB=tools/ablate/libpixpath_$lib.so timeout -k 10 200 python -u bench.py --allow-tuning \
          --workload config4 --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/occ_${lib}_${cho}_${rep}_$TAG.json \
          2>> gpurun_out/occ_$TAG.err || { tail -3 gpurun_out/occ_$TAG.err; exit 1; }
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['canvas_chain'];print('$lib cho $cho', $rep, c['avg_launch_ms'], c['frac'])" gpurun_out/occ_${lib}_${cho}_${rep}_$TAG.json
    done
  done
done
