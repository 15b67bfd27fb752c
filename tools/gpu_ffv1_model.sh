set -o pipefail
TAG=${1:-md}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ffv1.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_$TAG.log; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_$TAG.log | head -5
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$TAG -o run -- python3 bench.py --workload ffv1 --ffv1-concurrent 1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/kt_$TAG.log 2>&1 || exit 1
grep -E "ffv1" gpurun_out/kt_$TAG/run_kernel_stats.csv | cut -d, -f1,4
