# FFV1 decoder knob sweep (measurement build): lanes per wave, two-entry context cache.
set -o pipefail
TAG=${1:-sw}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/ffv1_dec_chunks.py 600 | tee gpurun_out/ffv1_sweep_$TAG.txt
. tools/ablate_env.sh
for cfg in "PIXPATH_FFV1_DC2=1" "PIXPATH_FFV1_LPW=8" "PIXPATH_FFV1_LPW=8 PIXPATH_FFV1_DC2=1" "PIXPATH_FFV1_LPW=12" "PIXPATH_FFV1_LPW=4 PIXPATH_FFV1_DC2=1"; do
  echo "$cfg $(env $cfg timeout -k 10 120 python -u tools/ffv1_dec_chunks.py 600)" | tee -a gpurun_out/ffv1_sweep_$TAG.txt || exit 1
done
