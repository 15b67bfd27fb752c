set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu_r1c.log 2>&1; echo "pytest rc=$?"
grep -E "passed|failed" gpurun_out/pytest_gpu_r1c.log | tail -3
timeout -k 10 300 python bench.py > gpurun_out/bench_r1a.json 2> gpurun_out/bench_r1a.err && cat gpurun_out/bench_r1a.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_kt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/prof_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/prof_write.log 2>&1
echo "final rc=$?"
find gpurun_out -name "*.csv" | head -20
