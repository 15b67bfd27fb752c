set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_cli.py tests/test_gpu_configs.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pt_chain.log 2>&1; rc=$?
tail -5 gpurun_out/pt_chain.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|mismatch" gpurun_out/pt_chain.log | head -20; exit $rc; fi
timeout -k 10 300 python -u tools/aux_kernels.py --frames 600 --launches 5 > gpurun_out/aux_chain.log 2>&1 && grep chain gpurun_out/aux_chain.log
