# Round 6 closing check: every GPU test, smoke, the default bench line.  usage: bash tools/gpu_check_r6.sh TAG
set -o pipefail
TAG=${1:-r6y}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu_$TAG.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));e=d['e2e_avpvs'];c=d['cpu_baseline'];print('value',d['value'],'frac',d['roofline']['frac'],'ms',d['roofline']['avg_launch_ms'],'siti',d['siti_kernel']['avg_launch_ms'],'cpu',c['value'],'e2e',e['frames_per_s'],e['single_pvs']['frames_per_s'],e.get('vs_cpu_e2e'))"
