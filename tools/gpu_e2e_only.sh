set -o pipefail
TAG=${1:-e2}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --pvs-total 8 --no-cpu-baseline --no-pipeline --no-siti-file > gpurun_out/bench_e2e_$TAG.json 2> gpurun_out/bench_e2e_$TAG.err || { tail -5 gpurun_out/bench_e2e_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_e2e_$TAG.json'));e=d.get('e2e_avpvs');print(e['frames_per_s'],e['seconds'],e['single_pvs']);print(e['stages'])"
