# round 4 session b: clamped V pass (strip/chain parity + config4 / config2
# lines), then the e2e shared/private encode-stream A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_scale.py tests/test_gpu_scale_long.py tests/test_gpu_ffv1.py > gpurun_out/r4b_pytest.log 2>&1 || { tail -30 gpurun_out/r4b_pytest.log; exit 1; }
tail -2 gpurun_out/r4b_pytest.log
timeout -k 10 300 python -u bench.py --workload config4 --steps 10 --warmup 3 > gpurun_out/r4b_c4.json 2> gpurun_out/r4b_c4.err || { tail -5 gpurun_out/r4b_c4.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r4b_c4.json'));c=d['canvas_chain'];print('chain', c['avg_launch_ms'], c['frac'], 'stall', d['roofline']['frac'])"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-pipeline --no-siti-file --no-e2e > gpurun_out/r4b_c2.json 2> gpurun_out/r4b_c2.err || { tail -5 gpurun_out/r4b_c2.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r4b_c2.json'));r=d['roofline'];print('strip', r['avg_launch_ms'], r['frac'], 'siti', d['siti_kernel']['avg_launch_ms'], 'value', d['value'])"
timeout -k 10 300 python -u bench.py --workload ffv1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4b_ffv1.json 2> gpurun_out/r4b_ffv1.err || { tail -5 gpurun_out/r4b_ffv1.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r4b_ffv1.json'));print('ffv1 enc', d['value'], 'dec', d['decode'], 'conc', d['concurrent'])"
bash tools/gpu_e2e_ab.sh
