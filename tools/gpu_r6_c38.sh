# Round 6: config-3 8-bit DIRECT lane-pair loads -- scaler tests, A/B vs a
# variant library, then FETCH_SIZE / WRITE_SIZE of the product.  usage: bash tools/gpu_r6_c38.sh TAG variant
set -o pipefail
TAG=$1; V=$2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_scale_long.py tests/test_gpu_configs.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/c38_pytest_$TAG.log 2>&1; rc=$?
tail -2 gpurun_out/c38_pytest_$TAG.log; grep -E "^(FAILED|ERROR)" gpurun_out/c38_pytest_$TAG.log | head
[ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
for rep in 1 2; do
  for lib in $PWD/tools/var/libpixpath_$V.so $PWD/processing-chain_amd/pixpath/libpixpath.so; do
    PIXPATH_LIB=$lib timeout -k 10 120 python3 bench.py --allow-tuning --workload config3-8 --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline --no-siti-file > gpurun_out/c38_$TAG.json 2> gpurun_out/c38_$TAG.err || { tail -3 gpurun_out/c38_$TAG.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/c38_$TAG.json'));r=d['roofline'];print('$(basename $lib)', r['avg_launch_ms'], r['frac'])"
  done
done
C38="--workload config3-8 --steps 2 --warmup 0 --pvs-total 2 --pool 2 --no-cpu-baseline --no-pipeline --no-siti-file"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/prof_c38${ctr}_$TAG -o run -- python3 bench.py $C38 > gpurun_out/prof_c38${ctr}_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_c38${ctr}_$TAG.log; exit 1; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_c38kt_$TAG -o run -- python3 bench.py --workload config3-8 --steps 4 --warmup 1 --no-cpu-baseline --no-pipeline --no-siti-file --pvs-total 4 --pool 4 > gpurun_out/prof_c38kt_$TAG.json 2> gpurun_out/prof_c38kt_$TAG.log || { tail -5 gpurun_out/prof_c38kt_$TAG.log; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/prof_c38FETCH_SIZE_$TAG/run_counter_collection.csv gpurun_out/prof_c38WRITE_SIZE_$TAG/run_counter_collection.csv gpurun_out/prof_c38kt_$TAG/run_kernel_trace.csv gpurun_out/pmc_traffic_config3-8_$TAG.json 600 > /dev/null || exit 1
python3 -c "import json;[print(k, v) for k,v in json.load(open('gpurun_out/pmc_traffic_config3-8_$TAG.json'))['kernels'].items()]"
