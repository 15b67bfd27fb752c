# One GPU session: parity tests, bench, rocprof kernel trace + PMC passes.
# Usage (through gpurun): bash tools/gpu_session.sh TAG [pytest targets]
set -o pipefail
TAG=${1:-run}
TESTS=${2:-tests}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest $TESTS -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"
tail -3 gpurun_out/pytest_gpu_$TAG.log
grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu_$TAG.log | head -20
# 0 = green, 1 = test failures: keep going; anything else (crash, abort, timeout) ends the call
if [ $rc -gt 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && cat gpurun_out/bench_$TAG.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 --pvs-per-rank 4 --no-cpu-baseline --no-pipeline > gpurun_out/prof_kt_$TAG.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch_$TAG -o run -- python3 bench.py --steps 2 --warmup 0 --pvs-per-rank 2 --no-cpu-baseline --no-pipeline > gpurun_out/prof_fetch_$TAG.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write_$TAG -o run -- python3 bench.py --steps 2 --warmup 0 --pvs-per-rank 2 --no-cpu-baseline --no-pipeline > gpurun_out/prof_write_$TAG.log 2>&1 &&
python3 tools/pmc_traffic.py gpurun_out/prof_fetch_$TAG/run_counter_collection.csv gpurun_out/prof_write_$TAG/run_counter_collection.csv gpurun_out/prof_kt_$TAG/run_kernel_trace.csv gpurun_out/pmc_traffic_$TAG.json 600 > /dev/null &&
grep -E "pp::" gpurun_out/prof_kt_$TAG/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
echo "final rc=$?"
