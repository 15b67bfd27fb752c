# FFV1 encode / decode rate per slice grid (bench --workload ffv1; 600 bench frames).
set -o pipefail
TAG=${1:-g}
mkdir -p gpurun_out
export TMPDIR=/tmp
for grid in 8x8 16x8 16x16; do
  timeout -k 10 300 python -u bench.py --workload ffv1 --ffv1-slices $grid --ffv1-concurrent 1 --steps 2 --warmup 1 > gpurun_out/ffv1_grid_${grid}_$TAG.json 2> gpurun_out/ffv1_grid_${grid}_$TAG.err || { tail -5 gpurun_out/ffv1_grid_${grid}_$TAG.err; exit 1; }
  echo "$grid $(cut -c1-900 gpurun_out/ffv1_grid_${grid}_$TAG.json)"
done
