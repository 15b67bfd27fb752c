set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pack.py tests/test_gpu_cli.py tests/test_stall_stream.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pt_pack.log 2>&1; rc=$?
tail -3 gpurun_out/pt_pack.log; grep -E "^(FAILED|ERROR)" gpurun_out/pt_pack.log | head -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/aux_kernels.py --out gpurun_out/aux_kernels.json 2>&1 | grep case
