# Config-4 chain: luma and chroma launches overlapped on two streams
# (PIXPATH_CHAIN_OVERLAP, measurement build) vs one stream, alternating, with
# the FUSE 9 / 11 instances.  Usage: bash tools/gpu_chain_ovl_r5.sh TAG
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
  for m in serial overlap; do
    if [ $m = overlap ]; then x="PIXPATH_CHAIN_OVERLAP=1"; else x=""; fi
    env $x PIXPATH_LIB=tools/ablate/libpixpath_ablate.so timeout -k 10 200 python -u bench.py --allow-tuning \
        --workload config4 --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/ovl_${m}_${rep}_$TAG.json \
        2>> gpurun_out/ovl_$TAG.err || { tail -3 gpurun_out/ovl_$TAG.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['canvas_chain'];print('$m', $rep, c['avg_launch_ms'], c['frac'])" gpurun_out/ovl_${m}_${rep}_$TAG.json
  done
done
