set -o pipefail
TAG=${1:-ov}
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do for ov in "" "--overlap"; do
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pipeline --no-siti-file --no-e2e $ov > gpurun_out/ov_${r}${ov}_$TAG.json 2>> gpurun_out/ov_$TAG.err || { tail -3 gpurun_out/ov_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ov_${r}${ov}_$TAG.json'));print('$ov', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['siti_kernel']['avg_launch_ms'])"
done; done
