# round 4, session a: FFV1 encoder rework (record budget, in-place resolve,
# packet buffer) -> FFV1 / CLI / config GPU tests, then the bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ffv1.py tests/test_gpu_cli.py tests/test_gpu_configs.py > gpurun_out/r4a_pytest.log 2>&1 || { tail -30 gpurun_out/r4a_pytest.log; exit 1; }
tail -3 gpurun_out/r4a_pytest.log
timeout -k 10 600 python -u bench.py > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err || { tail -20 gpurun_out/r4a_bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r4a_bench.json"))
e = d["e2e_avpvs"]
print("value", d["value"], "frac", d["roofline"]["frac"], "e2e", e["frames_per_s"], "single", e["single_pvs"]["frames_per_s"])
print("stages", json.dumps(e["stages"]))
print("single stages", json.dumps(e["single_pvs"]["stages"]))
print("pool", e["encoder_pool"], "vs_cpu", e.get("vs_cpu_e2e"), "cpu e2e", d["cpu_baseline"]["e2e"])
PY
