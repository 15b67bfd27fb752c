# A/B of cpvs workgroup size and stall unit order (measurement only)
set -o pipefail
for rep in 1 2; do
for v in "PIXPATH_CPVS_LANES=256" "PIXPATH_CPVS_LANES=64"; do
  echo "== $v"
  env $v timeout -k 10 300 python3 tools/aux_kernels.py --launches 5 2>&1 | grep case | python3 -c "import sys,json; [print('%-26s %.4f ms %.3f' % (d['case'], d['avg_launch_ms'], d['frac_of_8TBps'])) for d in map(json.loads, sys.stdin)]"
done
done
