# Round 6: e2e (single PVS + 4 PVS) A/B of a host-side env knob.  usage: bash tools/gpu_r6_e2e_ab.sh TAG VAR "v1 v2"
set -o pipefail
TAG=$1; VAR=$2; VALS=$3
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python3 bench.py --allow-tuning --steps 2 --warmup 1 --pvs-total 4 --pool 4 --no-pipeline --no-siti-file --cpu-seconds 2 --cpu-e2e-seconds 3 > gpurun_out/e2eab_${TAG}_${v}_$rep.json 2> gpurun_out/e2eab_${TAG}_${v}_$rep.err || { tail -5 gpurun_out/e2eab_${TAG}_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/e2eab_${TAG}_${v}_$rep.json'));e=d['e2e_avpvs'];s=e['single_pvs'];print('$VAR=$v e2e',e['frames_per_s'],'single',s['frames_per_s'],s['runs_s'],'lanes',s['stages']['lanes'])" || exit 1
  done
done
