set -o pipefail
TAG=${1:-cc}
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in 8x8 16x16; do for K in 2 4; do
  timeout -k 10 300 python -u bench.py --workload ffv1 --ffv1-slices $g --ffv1-concurrent $K --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ffv1c_${g}_${K}_$TAG.json 2>> gpurun_out/ffv1c_$TAG.err || { tail -5 gpurun_out/ffv1c_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ffv1c_${g}_${K}_$TAG.json'));print('$g K=$K single enc',d['value'],'dec',d['decode']['frames_per_s'],'| concurrent',d['concurrent'])"
done; done
