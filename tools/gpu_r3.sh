# Round-3 GPU session: all GPU tests, the bench line, a strip-width A/B
# (512 default vs PIXPATH_STRIP_TW=256), the FFV1 bench lines + kernel stats.
# Usage (through gpurun): bash tools/gpu_r3.sh TAG
set -o pipefail
TAG=${1:-r3}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu_$TAG.log | head -20
if [ $rc -gt 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print('value',d['value'],'frac',d['roofline']['frac'],'ms',d['roofline']['avg_launch_ms'],'siti',d['siti_kernel']['avg_launch_ms'],'e2e',d.get('e2e_avpvs',{}).get('frames_per_s'),'cpu',d['cpu_baseline']['value'])"
for tw in 256 512; do
  PIXPATH_STRIP_TW=$tw timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --pvs-total 64 --no-cpu-baseline --no-pipeline --no-siti-file --no-e2e > gpurun_out/ab_tw${tw}_$TAG.json 2>> gpurun_out/bench_$TAG.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab_tw${tw}_$TAG.json'));print('tw $tw', d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
  for wl in config3-10 config3-8; do
    PIXPATH_STRIP_TW=$tw timeout -k 10 200 python -u bench.py --workload $wl --steps 10 --warmup 2 --pvs-total 8 --no-cpu-baseline --no-pipeline > gpurun_out/ab_tw${tw}_${wl}_$TAG.json 2>> gpurun_out/bench_$TAG.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_tw${tw}_${wl}_$TAG.json'));print('tw $tw $wl', d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
  done
done
bash tools/gpu_ffv1_bench.sh $TAG
