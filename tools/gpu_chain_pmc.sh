# chain plan: parity, config-4 bench line (stall + canvas chain), PMC HBM bytes of the chain launch
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_cli.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pt_chain3.log 2>&1; rc=$?
tail -2 gpurun_out/pt_chain3.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" gpurun_out/pt_chain3.log | head; exit $rc; fi
timeout -k 10 200 python -u bench.py --workload config4 --steps 20 --warmup 3 > gpurun_out/bench_config4_v3.json 2> gpurun_out/bench_config4_v3.err && cat gpurun_out/bench_config4_v3.json &&
timeout -k 10 200 python -u tools/chain_ablate.py > gpurun_out/chain_ab_v3.log 2>&1 && cat gpurun_out/chain_ab_v3.log &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_chain -o run -- python3 tools/chain_ablate.py --frames 600 > gpurun_out/kt_chain.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_chain_fetch -o run -- python3 tools/chain_ablate.py --frames 600 > gpurun_out/pmc_chain_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_chain_write -o run -- python3 tools/chain_ablate.py --frames 600 > gpurun_out/pmc_chain_write.log 2>&1 &&
grep -E "strip_kernel|scale_kernel" gpurun_out/kt_chain/run_kernel_stats.csv | cut -d, -f1-5 | cut -c1-200
