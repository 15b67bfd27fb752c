# FFV1 coder ablation (timing only: PIXPATH_FFV1_DEBUG bits produce wrong output).
. tools/ablate_env.sh
set -o pipefail
TAG=${1:-ab}
mkdir -p gpurun_out
export TMPDIR=/tmp
for dbg in 0 1 2 4 7; do
  PIXPATH_FFV1_DEBUG=$dbg timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_ffv1_${dbg}_$TAG -o run -- python3 bench.py $BENCH_TUNE --workload ffv1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_ffv1_${dbg}_$TAG.log 2>&1 || true
  echo "debug $dbg: $(grep -E 'ffv1_code' gpurun_out/ab_ffv1_${dbg}_$TAG/run_kernel_stats.csv | cut -d, -f4)"
done
