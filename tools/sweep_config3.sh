# config-3 downscale plans: LDS budget / chunk height sweep (measurement only).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/sweep_config3.txt
: > $out
for wl in config3-10 config3-8; do
for cfg in "32 40" "32 56" "32 64" "32 80" "16 56" "16 64"; do
  set -- $cfg
  PIXPATH_SCALE_CHO_MAX=$1 PIXPATH_SCALE_LDS_KB=$2 \
    timeout -k 10 120 python bench.py --workload $wl --steps 8 --warmup 2 --pvs-per-rank 4 --no-cpu-baseline --no-pipeline > gpurun_out/sweep_one.json 2> gpurun_out/sweep_one.err || { tail -3 gpurun_out/sweep_one.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sweep_one.json')); print('%s cho<=%s lds=%sKB scale_ms=%.4f frac=%.3f' % (sys.argv[1], sys.argv[2], sys.argv[3], d['roofline']['avg_launch_ms'], d['roofline']['frac']))" $wl $1 $2 | tee -a $out
done
done
