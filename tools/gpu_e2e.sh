# e2e_avpvs only (bench config-2 line with the other extra legs off): stage
# accounting and per-PVS timeline of the GPU-FFV1 AVPVS path.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-e2e}
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pipeline --no-siti-file ${EXTRA} > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err || { tail -20 gpurun_out/${TAG}.err; exit 1; }
python3 - "$TAG" <<'PY'
import json, sys
d = json.load(open("gpurun_out/%s.json" % sys.argv[1]))
e = d["e2e_avpvs"]
print("e2e", e["frames_per_s"], "single", e["single_pvs"]["frames_per_s"], "pool", e["encoder_pool"])
for k in ("stages",):
    print(json.dumps(e[k]))
print(json.dumps(e["single_pvs"]["stages"]))
PY
