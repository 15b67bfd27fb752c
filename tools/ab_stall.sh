set -o pipefail
for rep in 1 2; do for g in 2 3 4 6; do
  echo -n "G=$g "; PIXPATH_STALL_G=$g timeout -k 10 300 python3 tools/aux_kernels.py --launches 5 2>&1 | grep stall_ | python3 -c "import sys,json; [print('%.4f ms %.3f' % (d['avg_launch_ms'], d['frac_of_8TBps'])) for d in map(json.loads, sys.stdin)]"
done; done
