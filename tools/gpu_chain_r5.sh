# Config-4 canvas chain (strip_kernel FUSE=10 chain plan) study, round 5:
# kernel trace of the product (luma launch / chroma launch apart), then the
# chroma segment count (PIXPATH_CHAIN_SEG2, measurement build) and chroma
# chunk-height variants (tools/build_variant.sh) on the same box.
# Usage (through gpurun): bash tools/gpu_chain_r5.sh TAG "variant ..."
set -o pipefail
TAG=$1; VARS=$2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_chain_$TAG -o run -- python3 bench.py --workload config4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/kt_chain_$TAG.json 2> gpurun_out/kt_chain_$TAG.err || { tail -5 gpurun_out/kt_chain_$TAG.err; exit 1; }
PIXPATH_TRACE_BY_GRID=1 python3 tools/trace_stats.py gpurun_out/kt_chain_$TAG/run_kernel_trace.csv 2 strip_kernel stall_kernel > gpurun_out/kt_chain_$TAG.csv
cut -d, -f1-5 gpurun_out/kt_chain_$TAG.csv | cut -c1-220
run() {  # name lib [env...]
  local v=$1 lib=$2; shift 2
  env "$@" PIXPATH_LIB=$lib timeout -k 10 120 python3 bench.py --allow-tuning --workload config4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/cv_${v}_$TAG.json 2> gpurun_out/cv_${v}_$TAG.err || { tail -3 gpurun_out/cv_${v}_$TAG.err; return 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/cv_${v}_$TAG.json'));c=d['canvas_chain'];print('$v', c['avg_launch_ms'], c['frac'])"
}
for rep in 1 2; do
  run product $PWD/processing-chain_amd/pixpath/libpixpath.so || exit 1
  for s in 2 8 16; do run seg$s $PWD/tools/ablate/libpixpath_ablate.so PIXPATH_CHAIN_SEG2=$s || exit 1; done
  run overlap $PWD/tools/ablate/libpixpath_ablate.so PIXPATH_CHAIN_OVERLAP=1 || exit 1
  run overlap_seg8 $PWD/tools/ablate/libpixpath_ablate.so PIXPATH_CHAIN_OVERLAP=1 PIXPATH_CHAIN_SEG2=8 || exit 1
  for v in $VARS; do run $v $PWD/tools/ablate/libpixpath_$v.so || exit 1; done
done
PIXPATH_CHAIN_OVERLAP=1 PIXPATH_LIB=$PWD/tools/ablate/libpixpath_ablate.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py > gpurun_out/cv_pytest_overlap_$TAG.log 2>&1; echo "overlap parity: $(tail -1 gpurun_out/cv_pytest_overlap_$TAG.log)"
for v in $VARS; do
  PIXPATH_LIB=$PWD/tools/ablate/libpixpath_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py > gpurun_out/cv_pytest_${v}_$TAG.log 2>&1; echo "$v parity: $(tail -1 gpurun_out/cv_pytest_${v}_$TAG.log)"
done
