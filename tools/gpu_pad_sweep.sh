# strip_kernel config 2 vs the output layout (pitch / frame-stride padding).
. tools/ablate_env.sh
set -o pipefail
TAG=${1:-pad}
mkdir -p gpurun_out
export TMPDIR=/tmp
for pp in "0 0" "256 0" "512 0" "0 1" "0 3" "128 1"; do
  set -- $pp
  PIXPATH_PITCH_PAD=$1 PIXPATH_ROWS_PAD=$2 timeout -k 10 120 python -u bench.py $BENCH_TUNE --steps 10 --warmup 2 --pvs-total 32 --no-cpu-baseline --no-pipeline --no-siti-file --no-e2e > gpurun_out/pad_$1_$2_$TAG.json 2>> gpurun_out/pad_$TAG.err || { tail -3 gpurun_out/pad_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/pad_$1_$2_$TAG.json'));print('pitch+$1 rows+$2', d['roofline']['avg_launch_ms'], d['roofline']['frac'], 'siti', d['siti_kernel']['avg_launch_ms'])"
done
