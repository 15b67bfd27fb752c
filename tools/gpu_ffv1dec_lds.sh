# FFV1 decoder with LDS-resident hot states: parity tests, then the 600-frame
# decode rate (product build), then slices per workgroup and the prologue
# ablation (measurement build; PIXPATH_FFV1_DEBUG output is wrong, timing only).
set -o pipefail
TAG=${1:-lds}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ffv1.py > gpurun_out/ffv1_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/ffv1_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/ffv1_tests_$TAG.log
timeout -k 10 120 python -u tools/ffv1_dec_chunks.py 600 60 | tee gpurun_out/ffv1_dec_$TAG.txt
. tools/ablate_env.sh
for l in; do
  echo "DPF=$l $(PIXPATH_FFV1_DPF=$l timeout -k 10 120 python -u tools/ffv1_dec_chunks.py 600)" | tee -a gpurun_out/ffv1_dec_$TAG.txt || exit 1
done
for dbg in; do
  echo "DEBUG=$dbg $(PIXPATH_FFV1_DEBUG=$dbg timeout -k 10 120 python -u tools/ffv1_dec_chunks.py 600)" | tee -a gpurun_out/ffv1_dec_$TAG.txt || exit 1
done
