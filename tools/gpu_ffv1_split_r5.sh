# FFV1 encode / decode time against the frames per batch (is a half batch's
# encode about half a full one's?), and the reference-shaped stream decode line.
# Usage: bash tools/gpu_ffv1_split_r5.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 600 300 150; do
  timeout -k 10 200 python -u bench.py --workload ffv1 --frames $n --steps 3 --warmup 1 --no-cpu-baseline \
      --ffv1-concurrent 1 > gpurun_out/ffv1_frames${n}_$TAG.json 2>> gpurun_out/ffv1_split_$TAG.err \
      || { tail -5 gpurun_out/ffv1_split_$TAG.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print($n, 'enc ms', d['ms_per_step'], 'dec ms', d['decode']['ms_per_step'], d['decode']['lossless'])" gpurun_out/ffv1_frames${n}_$TAG.json
done
timeout -k 10 400 python -u bench.py --workload ffv1 --steps 2 --warmup 1 --ffv1-concurrent 1 \
    > gpurun_out/ffv1_refdec_$TAG.json 2>> gpurun_out/ffv1_split_$TAG.err || { tail -5 gpurun_out/ffv1_split_$TAG.err; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(json.dumps(d.get('reference_stream_decode')))" gpurun_out/ffv1_refdec_$TAG.json
# kernel trace of the e2e_avpvs line (where do the extra ~20 ms per encode go?)
mkdir -p gpurun_out/e2e_trace_$TAG
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/e2e_trace_$TAG -o run -- \
    python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pipeline --no-siti-file \
    > gpurun_out/e2e_trace_$TAG.json 2>> gpurun_out/ffv1_split_$TAG.err || { tail -5 gpurun_out/ffv1_split_$TAG.err; exit 1; }
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));e=d['e2e_avpvs'];print('e2e', e['frames_per_s'], e['single_pvs']['frames_per_s'], e['single_pvs']['stages']['encode_s'])" gpurun_out/e2e_trace_$TAG.json
f=$(find gpurun_out/e2e_trace_$TAG -name '*kernel_stats.csv' | head -1); head -12 "$f"
