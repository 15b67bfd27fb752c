# Quick GPU iteration: scaler/SI-TI parity subset, bench line, rocprof kernel stats.
# Usage (through gpurun): bash tools/gpu_quick.sh TAG [pytest target] [bench args]
set -o pipefail
TAG=${1:-q}; T=${2:-tests/test_gpu_scale.py}; shift 2 2>/dev/null; BARGS="$@"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest $T -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/pt_$TAG.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error" gpurun_out/pt_$TAG.log | head; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 $BARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 --pvs-per-rank 8 --no-cpu-baseline --no-pipeline $BARGS > gpurun_out/kt_$TAG.log 2>&1 || { tail gpurun_out/kt_$TAG.log; exit 1; }
grep -E "pp::" gpurun_out/kt_$TAG/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
