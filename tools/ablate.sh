# Ablation of strip_kernel phases (timing only; outputs are wrong when debug != 0).
# bits: 1 no V stores, 2 no staging loads, 4 no H pass, 8 no barriers, 16 nontemporal stores
set -o pipefail
mkdir -p gpurun_out
for d in ${DEBUGS:-0 16 6 14 22 30 7}; do
  PIXPATH_SCALE_DEBUG=$d timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --pvs-per-rank 8 --no-cpu-baseline --no-pipeline $BARGS > gpurun_out/abl_$d.json 2>gpurun_out/abl_$d.err || { tail -3 gpurun_out/abl_$d.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/abl_$d.json')); print('debug=$d', d['roofline']['avg_launch_ms'], d.get('siti_kernel',{}).get('avg_launch_ms'))"
done
