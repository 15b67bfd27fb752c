set -o pipefail
TAG=${1:-rl}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ffv1.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_$TAG.log
if [ $rc -gt 1 ]; then exit $rc; fi
for r in 64 16 8; do
  PIXPATH_FFV1_RLPW=$r timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rl_${r}_$TAG -o run -- python3 bench.py --workload ffv1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/rl_${r}_$TAG.log 2>&1 || exit 1
  echo "rlpw $r: $(grep -E 'ffv1_resolve' gpurun_out/rl_${r}_$TAG/run_kernel_stats.csv | cut -d, -f4)"
done
