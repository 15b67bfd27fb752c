set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/chain_ablate.py > gpurun_out/chain_ab.log 2>&1 &&
PIXPATH_SCALE_CHO_MAX=16 timeout -k 10 120 python -u tools/chain_ablate.py >> gpurun_out/chain_ab.log 2>&1 &&
PIXPATH_SCALE_LDS_KB=64 timeout -k 10 120 python -u tools/chain_ablate.py >> gpurun_out/chain_ab.log 2>&1 &&
timeout -k 10 120 python -u tools/chain_ablate.py --src yuv420p --dst yuv422p >> gpurun_out/chain_ab.log 2>&1
cat gpurun_out/chain_ab.log | grep chain_ms
