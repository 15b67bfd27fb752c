# Config-4 chain, round 5: the product (split launches, paired second stage)
# against the combined single launch (PIXPATH_CHAIN_COMBINED) and chroma
# segment counts, per-launch kernel traces.
set -o pipefail
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
ABL=$PWD/tools/ablate/libpixpath_ablate.so
trace() {  # name lib [env ...]
  local v=$1 lib=$2; shift 2
  env "$@" PIXPATH_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_${v}_$TAG -o run -- python3 bench.py --allow-tuning --workload config4 --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/kt_${v}_$TAG.json 2> gpurun_out/kt_${v}_$TAG.err || { tail -3 gpurun_out/kt_${v}_$TAG.err; return 1; }
  echo "== $v $* $(python3 -c "import json;c=json.load(open('gpurun_out/kt_${v}_$TAG.json'))['canvas_chain'];print(c['avg_launch_ms'], c['frac'])")"
  PIXPATH_TRACE_BY_GRID=1 python3 tools/trace_stats.py gpurun_out/kt_${v}_$TAG/run_kernel_trace.csv 2 strip_kernel | cut -d, -f1,3,4 | tail -n +2
}
trace product $PWD/processing-chain_amd/pixpath/libpixpath.so || exit 1
trace combined $ABL PIXPATH_CHAIN_COMBINED=1 || exit 1
trace combined_seg2 $ABL PIXPATH_CHAIN_COMBINED=1 PIXPATH_CHAIN_SEG2=2 || exit 1
trace seg2 $ABL PIXPATH_CHAIN_SEG2=2 || exit 1
trace seg3 $ABL PIXPATH_CHAIN_SEG2=3 || exit 1
trace dbg16 $ABL PIXPATH_SCALE_DEBUG=16 || exit 1
PIXPATH_CHAIN_COMBINED=1 PIXPATH_LIB=$ABL timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py > gpurun_out/cv_pytest_combined_$TAG.log 2>&1; echo "combined parity: $(tail -1 gpurun_out/cv_pytest_combined_$TAG.log)"
