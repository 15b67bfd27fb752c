# Round-5 session: parity of the scaler paths touched (DIRECT H pass, chain
# segments), the config-3 lines, then the chain study.
# Usage (through gpurun): bash tools/gpu_r5_study.sh TAG "chain variants"
set -o pipefail
TAG=$1; VARS=$2
bash tools/gpu_r5.sh $TAG tests:"scale or chain or config or cli_avpvs" config3-8 config3-10 || exit 1
bash tools/gpu_chain_r5.sh $TAG "$VARS"
