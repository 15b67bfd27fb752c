# Round-6 session run for the judged artifacts: every GPU test, smoke, the
# bench line, a rocprof kernel trace (stats over the timed launches) + FETCH /
# WRITE PMC passes of the bench kernels, the config-4 chain (luma and chroma
# launches apart) and stall, config-3 8-bit traffic, the FFV1 line, config 3/4 lines.
# Usage (through gpurun): bash tools/gpu_final_r6.sh TAG
set -o pipefail
TAG=${1:-r6x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log; grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu_$TAG.log | head -20
if [ $rc -gt 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));e=d['e2e_avpvs'];c=d['cpu_baseline'];print('value',d['value'],'frac',d['roofline']['frac'],'ms',d['roofline']['avg_launch_ms'],'siti',d['siti_kernel']['avg_launch_ms'],'pcie',d.get('pcie_pipeline',{}).get('frames_per_s'),'cpu',c['value'],c['build'],'e2e',e['frames_per_s'],e['single_pvs']['frames_per_s'],e.get('vs_cpu_e2e'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 --pvs-total 4 --pool 4 --no-cpu-baseline --no-pipeline --no-siti-file --no-e2e > gpurun_out/prof_kt_$TAG.json 2> gpurun_out/prof_kt_$TAG.log || { tail -5 gpurun_out/prof_kt_$TAG.log; exit 1; }
python3 tools/trace_stats.py gpurun_out/prof_kt_$TAG/run_kernel_trace.csv 12 pp:: > gpurun_out/kernel_stats_timed_$TAG.csv
python3 -c "import json;d=json.load(open('gpurun_out/prof_kt_$TAG.json'));print('profiled run: strip avg_launch_ms', d['roofline']['avg_launch_ms'], 'siti', d['siti_kernel']['avg_launch_ms'])"
cut -d, -f1-8 gpurun_out/kernel_stats_timed_$TAG.csv | cut -c1-200
pmc() {  # name counter args...
  local n=$1 ctr=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/prof_${n}_$TAG -o run -- python3 bench.py "$@" > gpurun_out/prof_${n}_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_${n}_$TAG.log; return 1; }
}
B2="--steps 2 --warmup 0 --pvs-total 2 --pool 2 --no-cpu-baseline --no-pipeline --no-siti-file --no-e2e"
pmc fetch FETCH_SIZE $B2 && pmc write WRITE_SIZE $B2 || exit 1
python3 tools/pmc_traffic.py gpurun_out/prof_fetch_$TAG/run_counter_collection.csv gpurun_out/prof_write_$TAG/run_counter_collection.csv gpurun_out/prof_kt_$TAG/run_kernel_trace.csv gpurun_out/pmc_traffic_$TAG.json 600 > /dev/null || exit 1
C4="--workload config4 --steps 2 --warmup 1 --no-cpu-baseline"
C38="--workload config3-8 --steps 2 --warmup 0 --pvs-total 2 --pool 2 --no-cpu-baseline --no-pipeline --no-siti-file"
pmc c4fetch FETCH_SIZE $C4 && pmc c4write WRITE_SIZE $C4 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_c4kt_$TAG -o run -- python3 bench.py --workload config4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_config4_prof_$TAG.json 2> gpurun_out/prof_c4kt_$TAG.log || { tail -5 gpurun_out/prof_c4kt_$TAG.log; exit 1; }
PIXPATH_TRACE_BY_GRID=1 python3 tools/pmc_traffic.py gpurun_out/prof_c4fetch_$TAG/run_counter_collection.csv gpurun_out/prof_c4write_$TAG/run_counter_collection.csv gpurun_out/prof_c4kt_$TAG/run_kernel_trace.csv gpurun_out/pmc_traffic_config4_bygrid_$TAG.json 600 > /dev/null || exit 1
python3 tools/pmc_traffic.py gpurun_out/prof_c4fetch_$TAG/run_counter_collection.csv gpurun_out/prof_c4write_$TAG/run_counter_collection.csv gpurun_out/prof_c4kt_$TAG/run_kernel_trace.csv gpurun_out/pmc_traffic_config4_$TAG.json 600 > /dev/null || exit 1
PIXPATH_TRACE_BY_GRID=1 python3 tools/trace_stats.py gpurun_out/prof_c4kt_$TAG/run_kernel_trace.csv 2 pp:: > gpurun_out/kernel_stats_config4_$TAG.csv
pmc c38fetch FETCH_SIZE $C38 && pmc c38write WRITE_SIZE $C38 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_c38kt_$TAG -o run -- python3 bench.py --workload config3-8 --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline --no-siti-file --pvs-total 8 --pool 4 > gpurun_out/bench_config3-8_prof_$TAG.json 2> gpurun_out/prof_c38kt_$TAG.log || { tail -5 gpurun_out/prof_c38kt_$TAG.log; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/prof_c38fetch_$TAG/run_counter_collection.csv gpurun_out/prof_c38write_$TAG/run_counter_collection.csv gpurun_out/prof_c38kt_$TAG/run_kernel_trace.csv gpurun_out/pmc_traffic_config3-8_$TAG.json 600 > /dev/null || exit 1
python3 tools/trace_stats.py gpurun_out/prof_c38kt_$TAG/run_kernel_trace.csv 2 pp:: > gpurun_out/kernel_stats_config3-8_$TAG.csv
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_ffv1_$TAG -o run -- python3 bench.py --workload ffv1 --ffv1-concurrent 1 --steps 2 --warmup 1 > gpurun_out/bench_ffv1_$TAG.json 2> gpurun_out/bench_ffv1_$TAG.err || { tail -5 gpurun_out/bench_ffv1_$TAG.err; exit 1; }
grep -E "ffv1" gpurun_out/kt_ffv1_$TAG/run_kernel_stats.csv | cut -d, -f1-4
for wl in config3-10 config3-8 config4; do
  timeout -k 10 200 python -u bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-pipeline > gpurun_out/bench_${wl}_$TAG.json 2>> gpurun_out/bench_$TAG.err || { tail -3 gpurun_out/bench_$TAG.err; exit 1; }
  cut -c1-200 gpurun_out/bench_${wl}_$TAG.json
done
python3 -c "import json;[print(k, round(v['hbm_bytes_per_launch']/1e9,3), 'GB', v['avg_duration_ns']) for f in ['pmc_traffic_$TAG','pmc_traffic_config4_bygrid_$TAG','pmc_traffic_config4_$TAG','pmc_traffic_config3-8_$TAG'] for k,v in json.load(open('gpurun_out/'+f+'.json'))['kernels'].items()]"
