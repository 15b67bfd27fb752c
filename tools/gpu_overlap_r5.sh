# config-2 bench line with and without --overlap (SI/TI on a second stream),
# alternating.  Usage: bash tools/gpu_overlap_r5.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for m in plain overlap; do
    if [ $m = overlap ]; then o=--overlap; else o=""; fi
    timeout -k 10 200 python -u bench.py $o --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline --no-siti-file --no-e2e \
        > gpurun_out/ov_${m}_${rep}_$TAG.json 2>> gpurun_out/ov_$TAG.err || { tail -3 gpurun_out/ov_$TAG.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print('$m', $rep, d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], d.get('siti_kernel',{}).get('avg_launch_ms'))" gpurun_out/ov_${m}_${rep}_$TAG.json
  done
done
