# Config-3 8-bit (strip_kernel DIRECT) chunk-height study, round 5: the
# measurement build's PIXPATH_SCALE_CHO_MAX / PIXPATH_SCALE_LDS_KB let the plan
# take taller chunks (the DIRECT launch's LDS is the V window ring only).
set -o pipefail
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
ABL=$PWD/tools/ablate/libpixpath_ablate.so
run() {  # name lib [env ...]
  local v=$1 lib=$2; shift 2
  env "$@" PIXPATH_LIB=$lib timeout -k 10 120 python3 bench.py --allow-tuning --workload config3-8 --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline --no-siti-file --pvs-total 16 --pool 4 > gpurun_out/c38_${v}_$TAG.json 2> gpurun_out/c38_${v}_$TAG.err || { tail -3 gpurun_out/c38_${v}_$TAG.err; return 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/c38_${v}_$TAG.json'));r=d['roofline'];print('$v', r['avg_launch_ms'], r['frac'], r['plan'])"
}
for rep in 1 2; do
  run product $PWD/processing-chain_amd/pixpath/libpixpath.so || exit 1
  run cho16 $ABL PIXPATH_SCALE_CHO_MAX=16 PIXPATH_SCALE_LDS_KB=96 || exit 1
  run cho24 $ABL PIXPATH_SCALE_CHO_MAX=24 PIXPATH_SCALE_LDS_KB=128 || exit 1
  run cho32 $ABL PIXPATH_SCALE_CHO_MAX=32 PIXPATH_SCALE_LDS_KB=160 || exit 1
done
PIXPATH_SCALE_CHO_MAX=32 PIXPATH_SCALE_LDS_KB=160 PIXPATH_LIB=$ABL timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_scale.py tests/test_gpu_scale_long.py > gpurun_out/c38_pytest_$TAG.log 2>&1; echo "cho32 parity: $(tail -1 gpurun_out/c38_pytest_$TAG.log)"
