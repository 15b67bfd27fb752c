# counter passes on the config-3 8-bit strip plan (isolated launches) and the config-2 plan for comparison
set -o pipefail
PK_ARGS="--src yuv420p:3840x2160 --flags bicubic --frames 300" bash tools/gpu_counters.sh c38 scale > gpurun_out/ctr_c38.txt 2>&1; rc=$?; tail -45 gpurun_out/ctr_c38.txt; exit $rc
