# kernel + memory-copy timeline of the e2e_avpvs leg (no PMC counters).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/e2etrace
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/e2etrace -- python3 -u bench.py --steps 1 --warmup 0 --pvs-total 4 --no-cpu-baseline --no-pipeline --no-siti-file > gpurun_out/e2etrace.json 2> gpurun_out/e2etrace.err || { tail -20 gpurun_out/e2etrace.err; exit 1; }
python3 tools/e2e_trace.py gpurun_out/e2etrace 1.6 > gpurun_out/e2etrace_summary.txt
python3 -c "import json;d=json.load(open('gpurun_out/e2etrace.json'));e=d['e2e_avpvs'];print(e['frames_per_s'], e['single_pvs']['frames_per_s']);print(json.dumps(e['stages']))"
head -c 3000 gpurun_out/e2etrace_summary.txt
