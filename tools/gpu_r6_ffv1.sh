# Round 6: FFV1 writer lanes + group decode + e2e (split 2 vs 1).  usage: bash tools/gpu_r6_ffv1.sh TAG
set -o pipefail
TAG=${1:-r6f}
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests/test_gpu_ffv1.py tests/test_gpu_ffv1_general.py tests/test_gpu_cli.py tests/test_gpu_configs.py tests/test_gpu_pack.py}
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ffv1_pytest_$TAG.log 2>&1; rc=$?
tail -2 gpurun_out/ffv1_pytest_$TAG.log; grep -E "^(FAILED|ERROR)" gpurun_out/ffv1_pytest_$TAG.log | head
[ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
[ -z "$NOFFV1BENCH" ] && { timeout -k 10 400 python3 bench.py --workload ffv1 --steps 2 --warmup 1 > gpurun_out/bench_ffv1_$TAG.json 2> gpurun_out/bench_ffv1_$TAG.err || { tail -5 gpurun_out/bench_ffv1_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_ffv1_$TAG.json'));print('ffv1 enc',d['value'],'dec',d['decode']['frames_per_s'],'lanes',d.get('writer_lanes'));r=d.get('reference_stream_decode') or {};print('refdec',json.dumps({k:r.get(k) for k in ('streams','cpu_oracle','cpu_oracle_16','gpu_best_vs_cpu_16')}))" || exit 1; }
for sp in ${SPLITS:-3 2 1}; do
  if [ $sp = auto ]; then unset PIXPATH_FFV1_SPLIT; else export PIXPATH_FFV1_SPLIT=$sp; fi
  timeout -k 10 400 python3 bench.py --steps 2 --warmup 1 --pvs-total 4 --pool 4 --no-pipeline --no-siti-file --cpu-seconds 4 --cpu-e2e-seconds 4 > gpurun_out/bench_e2e_s${sp}_$TAG.json 2> gpurun_out/bench_e2e_s${sp}_$TAG.err || { tail -5 gpurun_out/bench_e2e_s${sp}_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_e2e_s${sp}_$TAG.json'));e=d['e2e_avpvs'];print('split $sp e2e',e['frames_per_s'],'single',e['single_pvs']['frames_per_s'],e['single_pvs']['runs_s'],'vs_cpu',e.get('vs_cpu_e2e'),'timeline',e['single_pvs']['stages']['timeline'],'lanes',e['stages'].get('writer_lanes'))" || exit 1
done
