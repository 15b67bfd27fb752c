# Round-5 GPU session steps (run through gpurun).  Every GPU step has its own
# time limit; the script stops at the first failure.
# Usage: bash tools/gpu_r5.sh TAG STEP [STEP ...]
#   tests           every -m gpu test
#   tests:<expr>    -m gpu tests selected with -k <expr>
#   smoke           __graft_entry__.smoke()
#   bench           default bench line (config 2 / 5)
#   config4|config3-8|config3-10|ffv1   the other workload lines
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
      echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu_$TAG.log | head -20
      if [ $rc -gt 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi ;;
    tests:*)
      timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "${step#tests:}" > gpurun_out/pytest_sel_$TAG.log 2>&1; rc=$?
      echo "pytest(${step#tests:}) rc=$rc"; tail -2 gpurun_out/pytest_sel_$TAG.log; grep -E "^(FAILED|ERROR)|Error" gpurun_out/pytest_sel_$TAG.log | head -20
      if [ $rc -gt 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi ;;
    smoke)
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
      tail -1 gpurun_out/smoke_$TAG.log ;;
    bench)
      timeout -k 10 500 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
      cut -c1-600 gpurun_out/bench_$TAG.json ;;
    config4|config3-8|config3-10)
      timeout -k 10 200 python -u bench.py --workload $step --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/bench_${step}_$TAG.json 2>> gpurun_out/bench_$TAG.err || { tail -3 gpurun_out/bench_$TAG.err; exit 1; }
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print('$step', d['value'], r['avg_launch_ms'], r['frac'], 'chain' if 'canvas_chain' in d else '', d.get('canvas_chain',{}).get('avg_launch_ms'), d.get('canvas_chain',{}).get('frac'))" gpurun_out/bench_${step}_$TAG.json ;;
    ffv1)
      timeout -k 10 300 python -u bench.py --workload ffv1 --steps 2 --warmup 1 > gpurun_out/bench_ffv1_$TAG.json 2>> gpurun_out/bench_$TAG.err || { tail -3 gpurun_out/bench_$TAG.err; exit 1; }
      cut -c1-800 gpurun_out/bench_ffv1_$TAG.json ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
