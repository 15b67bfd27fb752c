# A/B of chain-kernel library variants (tools/build_variant.sh) on the config-4
# canvas launch; parity of the product build first.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py > gpurun_out/cv_pytest.log 2>&1 || { tail -20 gpurun_out/cv_pytest.log; exit 1; }
tail -1 gpurun_out/cv_pytest.log
for rep in 1 2; do
for v in head product words cho24 cho32; do
  if [ $v = product ]; then lib=$PWD/processing-chain_amd/pixpath/libpixpath.so; else lib=$PWD/tools/ablate/libpixpath_$v.so; fi
  PIXPATH_LIB=$lib timeout -k 10 120 python3 bench.py --allow-tuning --workload config4 --steps 10 --warmup 3 > gpurun_out/cv_$v.json 2> gpurun_out/cv_$v.err || { tail -3 gpurun_out/cv_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/cv_$v.json'));c=d['canvas_chain'];print('$v', c['avg_launch_ms'], c['frac'])"
done
done
for v in cho24 cho32; do
  PIXPATH_LIB=$PWD/tools/ablate/libpixpath_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py > gpurun_out/cv_pytest_$v.log 2>&1; echo "$v parity: $(tail -1 gpurun_out/cv_pytest_$v.log)"
done
