set -o pipefail
for pc in ${PCS:-6 5 4 7}; do
  PIXPATH_SCALE_PER_CU=$pc timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --pvs-per-rank 8 --no-cpu-baseline --no-pipeline > gpurun_out/pc.json 2>gpurun_out/pc.err || { tail -3 gpurun_out/pc.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/pc.json')); print('per_cu=$pc', d['roofline']['avg_launch_ms'])"
done
