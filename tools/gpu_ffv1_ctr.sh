# FFV1 coder counters: one bench --workload ffv1 step per PMC pass (each pass
# its own rocprofv3 run), summarised per kernel.  Usage: bash tools/gpu_ffv1_ctr.sh TAG
set -o pipefail
TAG=${1:-ctr}
mkdir -p gpurun_out/ctr_$TAG
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/ctr_$TAG/p$i -o run -- python3 bench.py --workload ffv1 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/ctr_$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/ctr_$TAG/p$i.log; exit 1; }
done
python3 tools/summarize_counters.py gpurun_out/ctr_$TAG
