# Split-state decoder timing ablation (measurement build; the output is wrong):
# PIXPATH_FFV1_DEBUG 8 = no hot-half loads, 16 = no hot-half stores, 24 = neither.
set -o pipefail
TAG=${1:-ab}
mkdir -p gpurun_out
export TMPDIR=/tmp
. tools/ablate_env.sh
for dbg in 0 8 16 24; do
  echo "DEBUG=$dbg $(PIXPATH_FFV1_DEBUG=$dbg timeout -k 10 120 python -u tools/ffv1_dec_chunks.py 600 60)" | tee -a gpurun_out/ffv1_ablate2_$TAG.txt || exit 1
done
