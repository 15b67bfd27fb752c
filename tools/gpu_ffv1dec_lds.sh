# FFV1 decoder A/B step: the FFV1 GPU parity tests, then the 600-frame decode
# time as one launch and as ten 60-frame launches (tools/ffv1_dec_chunks.py;
# product build).  Usage (through gpurun): bash tools/gpu_ffv1dec_lds.sh TAG
set -o pipefail
TAG=${1:-lds}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ffv1.py > gpurun_out/ffv1_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/ffv1_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/ffv1_tests_$TAG.log
timeout -k 10 120 python -u tools/ffv1_dec_chunks.py 600 60 | tee gpurun_out/ffv1_dec_$TAG.txt
