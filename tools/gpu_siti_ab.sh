# SI/TI scheduling A/B: parity, same-box timing vs tools/libvariants, FETCH/WRITE traffic of the current library.
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_siti.sh || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sab_kt -o run -- python3 bench.py --steps 2 --warmup 0 --pvs-per-rank 2 --no-cpu-baseline --no-pipeline > gpurun_out/sab_kt.log 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/sab_fetch -o run -- python3 bench.py --steps 2 --warmup 0 --pvs-per-rank 2 --no-cpu-baseline --no-pipeline > gpurun_out/sab_fetch.log 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/sab_write -o run -- python3 bench.py --steps 2 --warmup 0 --pvs-per-rank 2 --no-cpu-baseline --no-pipeline > gpurun_out/sab_write.log 2>&1 &&
python3 tools/pmc_traffic.py gpurun_out/sab_fetch/run_counter_collection.csv gpurun_out/sab_write/run_counter_collection.csv gpurun_out/sab_kt/run_kernel_trace.csv gpurun_out/pmc_traffic_sab.json 600 > /dev/null &&
python3 -c "import json; d=json.load(open('gpurun_out/pmc_traffic_sab.json'))['kernels']; print({k: (v['hbm_bytes_per_launch'], v['avg_duration_ns']) for k, v in d.items()})"
