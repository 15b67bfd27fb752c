# strip_kernel counters: config-2 plan and config-4 chain plan, one rocprofv3
# run per PMC pass.  Usage: bash tools/gpu_strip_ctr.sh TAG
set -o pipefail
TAG=${1:-sc}
export TMPDIR=/tmp
for wl in config4 config2; do
  mkdir -p gpurun_out/sctr_${wl}_$TAG
  i=0
  if [ $wl = config2 ]; then ARGS="--steps 1 --warmup 0 --pvs-total 2 --pool 2 --no-cpu-baseline --no-pipeline --no-siti-file --no-e2e"; else ARGS="--workload config4 --steps 1 --warmup 0 --no-cpu-baseline"; fi
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
             "SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/sctr_${wl}_$TAG/p$i -o run -- python3 bench.py $ARGS > gpurun_out/sctr_${wl}_$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/sctr_${wl}_$TAG/p$i.log; exit 1; }
  done
  echo "### $wl"; python3 tools/summarize_counters.py gpurun_out/sctr_${wl}_$TAG | grep -A20 "strip_kernel"
done
