# FFV1 encoder with split hot/cold context states: the FFV1 GPU tests (packets
# byte-identical to the C restatement), then the FFV1 bench line.
set -o pipefail
TAG=${1:-enc}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ffv1.py > gpurun_out/ffv1enc_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/ffv1enc_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/ffv1enc_tests_$TAG.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_ffv1enc_$TAG -o run -- python3 bench.py --workload ffv1 --ffv1-concurrent 1 --steps 2 --warmup 1 > gpurun_out/bench_ffv1enc_$TAG.json 2> gpurun_out/bench_ffv1enc_$TAG.err || { tail -5 gpurun_out/bench_ffv1enc_$TAG.err; exit 1; }
cut -c1-700 gpurun_out/bench_ffv1enc_$TAG.json
grep -E "ffv1" gpurun_out/kt_ffv1enc_$TAG/run_kernel_stats.csv | cut -d, -f1-4
