# Config-4 chain, round 5 (split launches): per-launch kernel traces of the
# product, of measurement-build variants (one launch; 270-row luma segments)
# and of the timing ablation bits (PIXPATH_SCALE_DEBUG: 1 no V-pass stores,
# 2 no staging loads, 4 no H pass, 8 no barriers, 16 no second stage).
# Usage (through gpurun): bash tools/gpu_chain_r5b.sh TAG
set -o pipefail
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
ABL=$PWD/tools/ablate/libpixpath_ablate.so
trace() {  # name lib [env ...]
  local v=$1 lib=$2; shift 2
  env "$@" PIXPATH_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_${v}_$TAG -o run -- python3 bench.py --allow-tuning --workload config4 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/kt_${v}_$TAG.json 2> gpurun_out/kt_${v}_$TAG.err || { tail -3 gpurun_out/kt_${v}_$TAG.err; return 1; }
  echo "== $v $*"
  PIXPATH_TRACE_BY_GRID=1 python3 tools/trace_stats.py gpurun_out/kt_${v}_$TAG/run_kernel_trace.csv 2 strip_kernel | cut -d, -f1,3,4 | tail -n +2
}
trace product $PWD/processing-chain_amd/pixpath/libpixpath.so || exit 1
trace onelaunch $ABL PIXPATH_CHAIN_ONE_LAUNCH=1 || exit 1
trace luma270 $ABL PIXPATH_SCALE_SEG_ROWS=270 || exit 1
trace seg2_luma270 $ABL PIXPATH_SCALE_SEG_ROWS=270 PIXPATH_CHAIN_SEG2=2 || exit 1
for d in 1 2 4 8 16 6 22; do trace dbg$d $ABL PIXPATH_SCALE_DEBUG=$d || exit 1; done
